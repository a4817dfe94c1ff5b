// Diagnostic (bench.py's roofline, not on the codec path): the v_mfma_f32_16x16x32_bf16 rate this
// device sustains on random operands.  The chip lowers its clock under dense MFMA load, more on
// random data than on zeros (MI355X_MICROARCH.md "DVFS give-back"), so the dense-BF16 spec peak
// (2.5 PFLOP/s at 2.4 GHz) is not reachable by any kernel; this loop measures the ceiling that is:
// operands in registers (no LDS, no memory; the A operands re-randomised every iteration), eight
// independent accumulators per wave, four waves per SIMD, every CU busy.
#include "bc_common.h"
#include "x6_common.h"

namespace bc {

__global__ void __launch_bounds__(256, 4) mfma_probe_kernel(float* out, int iters, unsigned seed) {
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8_t a[2], b[4];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      a[k][e] = (__bf16)((float)(splitmix64(seed ^ (tid * 64ull + k * 8 + e)) >> 40) * 0x1p-24f - 0.5f);
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      b[k][e] = (__bf16)((float)(splitmix64(~seed ^ (tid * 64ull + k * 8 + e)) >> 40) * 0x1p-24f - 0.5f);
  floatx4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  // the A operands change every iteration (xor with a random per-lane mask, one VALU op per MFMA)
  // so the matrix pipes see fresh random data, as in a real GEMM loop, not one held pattern
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const u32x4_t m = {(unsigned)splitmix64(seed + tid), (unsigned)splitmix64(seed + tid + 1),
                     (unsigned)splitmix64(seed + tid + 2), (unsigned)splitmix64(seed + tid + 3)};
  for (int it = 0; it < 2 * iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 1], b[i & 3], acc[i], 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 2; ++k) a[k] = __builtin_bit_cast(bf16x8_t, __builtin_bit_cast(u32x4_t, a[k]) ^ m);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if ((threadIdx.x & 63) == 0) out[tid >> 6] = s;
}

// 16 MFMAs per iteration per wave; nwg workgroups of 4 waves.  out: nwg * 4 floats.
int mfma_probe_launch(float* out, int nwg, int iters, hipStream_t st) {
  if (!out || nwg <= 0 || iters <= 0) return BC_ERR_ARG;
  hipLaunchKernelGGL(mfma_probe_kernel, dim3(nwg), dim3(256), 0, st, out, iters, 0x5eedu);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

}  // namespace bc
