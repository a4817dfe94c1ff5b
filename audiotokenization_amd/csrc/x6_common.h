// Shared pieces of the 3xbf16 ("x6") MFMA kernels: conv1d_x6.hip (one conv per launch) and
// resunit_x6.hip (a whole ResidualUnit per launch).  See conv1d_x6.hip for the arithmetic.
#pragma once
#include <cstddef>

#include "bc_common.h"
#include "bc_internal.h"

namespace bc {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_void_t;

constexpr int X6_BKC = 32;            // channels per chunk = K of one bf16 MFMA
constexpr int X6_PITCH = 80;          // bytes per column per plane (64 data + 16 pad)
constexpr int X6_MAXCOL_ITERS = 11;   // 32-column passes per chunk: NCOL <= 352 (22 B loads / thread)

// s_waitcnt vmcnt(N) with the other counters left alone (gfx9 encoding: vmcnt[3:0] + [15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const bf16x2_t v = __builtin_convertvector((float2_t){a, b}, bf16x2_t);
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ float bf_lo(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bf_hi(unsigned p) { return __uint_as_float(p & 0xffff0000u); }

// exact split of two fp32 values into three packed bf16x2 planes: v = h + m + l
__device__ __forceinline__ void split2(float v0, float v1, unsigned& h, unsigned& m, unsigned& l) {
  h = pk_bf16(v0, v1);
  const float r0 = v0 - bf_lo(h), r1 = v1 - bf_hi(h);
  m = pk_bf16(r0, r1);
  const float s0 = r0 - bf_lo(m), s1 = r1 - bf_hi(m);
  l = pk_bf16(s0, s1);
}

// host-side tile geometry
struct X6Tile {
  int MT, NT, WM, WN;
};
inline int x6_BM(const X6Tile& t) { return 16 * t.MT * t.WM; }
inline int x6_BN(const X6Tile& t) { return 16 * t.NT * t.WN; }
inline int x6_ncol(const X6Tile& t, int K, int s, int d) { return (x6_BN(t) - 1) * s + (K - 1) * d + 1; }
const X6Tile& x6_tile(int cfg);  // cfg 100.. / 200.. -> tile (conv1d_x6.hip)

}  // namespace bc
