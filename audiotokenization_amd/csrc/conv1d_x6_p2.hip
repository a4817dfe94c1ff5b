// h3 (2 fp16 planes) instantiations of the conv kernel (conv1d_x6_kernel.h): one
// translation unit per precision so the library builds in parallel.
#include "conv1d_x6_kernel.h"

namespace bc {
template <>
int x6_launch_tile<2>(ConvArgs& a, int B, int tile, hipStream_t st) {
  BC_X6_TILE_SWITCH(2)
}
}  // namespace bc

BC_DEBUG_EXPORT(conv1d_x6_p2)
