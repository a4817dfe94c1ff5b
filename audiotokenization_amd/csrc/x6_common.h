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
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

constexpr int X6_BKC = 32;            // channels per chunk = K of one bf16 MFMA
constexpr int X6_PITCH = 80;          // bytes per column per plane (64 data + 16 pad)
// conv1d_x6_kernel's B tile: stride-1 tiles use a 64-B pitch with the four 16-B channel groups of
// column c XOR-swizzled by (c >> 1) & 3 (conflict-free ds_read_b128 fragment reads at any tap shift,
// 4-way ds_write_b32 staging); strided tiles keep the padded 80-B pitch (conflict-free at stride 2).
inline int x6_pitch(int s) { return s == 1 ? 64 : 80; }
constexpr int X6_MAXCOL_ITERS = 11;   // 32-column passes per chunk: NCOL <= 352 (22 B loads / thread)

// s_waitcnt vmcnt(N) with the other counters left alone (gfx9 encoding: vmcnt[3:0] + [15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// Issue-order pin between an LDS-DMA copy (global_load_lds) and the input loads that follow it: the
// counted `wait_vmcnt<N>` after those N loads retires the copy only if every one of them is issued AFTER
// it (vmcnt retires in issue order).  LDS and global memory do not alias, so nothing else stops LLVM from
// hoisting a buffer load above the copy: the empty asm with a memory clobber fences the IR passes, the
// sched_barrier the machine scheduler.  tools/check_vmcnt.py audits the built ISA for it.
__device__ __forceinline__ void dma_issue_order() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
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

// ---- "h3" operands (precision mode 3): two fp16 planes per fp32 value, three products ----
// v*S = h + m with h = fp16_rn(v*S), m = fp16_rn(v*S - h) (the residual v*S - h is exact in fp32), so
// |v*S - h - m| <= 2^-22 |v*S|; a*b is accumulated as a0b0 + a0b1 + a1b0 (a1b1 <= 2^-22 |ab| dropped).
// fp16 has 11 significant bits (3 more than bf16) but a 5-bit exponent, so every operand block is
// scaled by a power of two S = 2^(14 - e) with 2^e <= amax < 2^(e+1): |v*S| < 2^15 < 65504, and an
// element far below amax only loses precision that is negligible against amax (the dot-product
// scale): its absolute error stays below 2^-25 / S = 2^-39 amax.  Scaling by 2^k is exact, so the
// fp32 MFMA accumulation of the scaled products is the scaled accumulation of the unscaled ones.
__device__ __forceinline__ unsigned pk_f16(float a, float b) {
  const f16x2_t v = __builtin_convertvector((float2_t){a, b}, f16x2_t);
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ float f16_lo(unsigned p) {
  return (float)__builtin_bit_cast(f16x2_t, p)[0];
}
__device__ __forceinline__ float f16_hi(unsigned p) {
  return (float)__builtin_bit_cast(f16x2_t, p)[1];
}
// split of two (already scaled) fp32 values into two packed fp16x2 planes
__device__ __forceinline__ void split2_h(float v0, float v1, unsigned& h, unsigned& m) {
  h = pk_f16(v0, v1);
  m = pk_f16(v0 - f16_lo(h), v1 - f16_hi(h));
}
// exponent e of a block maximum (bits of a non-negative float) -> scale 2^(14 - e), clamped to a
// normal fp32; an all-zero block gets 1
__device__ __forceinline__ float h3_scale_from_bits(unsigned amax_bits) {
  int e = (int)(amax_bits >> 23) - 127;
  if (amax_bits == 0) e = 14;
  e = e < -112 ? -112 : (e > 140 ? 140 : e);
  return __uint_as_float((unsigned)(127 + 14 - e) << 23);
}
// max over the 64 lanes of a wave (non-negative float bits compare as unsigned ints)
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned w = (unsigned)__shfl_xor((int)v, o, 64);
    v = v > w ? v : w;
  }
  return v;
}

template <int P> struct FragType { typedef bf16x8_t type; };
template <> struct FragType<2> { typedef f16x8_t type; };

// host-side tile geometry
struct X6Tile {
  int MT, NT, WM, WN;
};
inline int x6_BM(const X6Tile& t) { return 16 * t.MT * t.WM; }
inline int x6_BN(const X6Tile& t) { return 16 * t.NT * t.WN; }
inline int x6_ncol(const X6Tile& t, int K, int s, int d) { return (x6_BN(t) - 1) * s + (K - 1) * d + 1; }
const X6Tile& x6_tile(int cfg);  // cfg 100.. / 200.. -> tile (conv1d_x6.hip)

}  // namespace bc
