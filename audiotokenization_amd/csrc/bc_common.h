// Shared device helpers for the BigCodec gfx950 kernels.
//
// Every kernel in this library computes in fp32.  The whole library is compiled with
// -ffp-contract=off so that elementwise expressions round exactly where the reference's torch
// expressions round (an explicit fmaf() is used wherever a fused multiply-add is intended).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define BC_OK 0
#define BC_ERR_ARG 1
#define BC_ERR_LAUNCH 2
#define BC_ERR_UNSUPPORTED 3

#define BC_CHECK_LAUNCH()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return BC_ERR_LAUNCH;             \
  } while (0)

// Ablation switches (tools/*_ablation.sh timing experiments that deliberately skip work) exist only in
// builds with -DBC_ABLATION; in the product library BC_ABL is the constant 0 and the branches vanish.
#ifdef BC_ABLATION
#define BC_ABL(flags, bit) ((flags) & (bit))
#else
#define BC_ABL(flags, bit) 0
#endif

// Bounds-checked debug build: `-DBC_DEBUG` (build_lib.build(debug=True) ->
// libbigcodec_hip_debug.so, loaded when BIGCODEC_DEBUG=1).  BC_DOK(cond) guards a global access whose index a
// kernel computed (epilogue stores and residual reads, weight copies, the LSTM's hand-off slots): a failed check
// counts into this translation unit's bc_dbg_word (failures, first failing source line) with vector atomics and
// the access is SKIPPED, so the kernel cannot fault; bc_debug_status() (abi.hip) reads and clears every unit's
// words.  In the product library BC_DOK is the constant true and the guards vanish.
#ifdef BC_DEBUG
namespace bc {
static __device__ unsigned bc_dbg_word[2];
__device__ __noinline__ static bool bc_dbg_fail(unsigned line) {
  atomicAdd(&bc_dbg_word[0], 1u);
  atomicCAS(&bc_dbg_word[1], 0u, line);
  return false;
}
}  // namespace bc
#define BC_DOK(cond) ((cond) ? true : ::bc::bc_dbg_fail(__LINE__))
// host reader of this translation unit's words (read and cleared; out[0] failures, out[1] first line)
#define BC_DEBUG_EXPORT(tu)                                                                       \
  extern "C" int bc_dbg_fetch_##tu(unsigned* out) {                                               \
    unsigned w[2] = {0, 0};                                                                       \
    if (hipMemcpyFromSymbol(w, HIP_SYMBOL(::bc::bc_dbg_word), sizeof(w)) != hipSuccess) return 2; \
    const unsigned z[2] = {0, 0};                                                                 \
    if (hipMemcpyToSymbol(HIP_SYMBOL(::bc::bc_dbg_word), z, sizeof(z)) != hipSuccess) return 2;   \
    out[0] += w[0];                                                                               \
    if (!out[1]) out[1] = w[1];                                                                   \
    return 0;                                                                                     \
  }
#else
#define BC_DOK(cond) true
#define BC_DEBUG_EXPORT(tu)
#endif

namespace bc {

// sin(x) for the Snake: Cody-Waite reduction by pi in 4 fma steps (valid for |x| < 39000), odd
// degree-9 minimax polynomial on [-pi/2, pi/2] -- the published SLEEF xsinf (u3.5) algorithm and
// constants -- about 20 instructions instead of OCML sinf's ~150 with its Payne-Hanek path.  Inputs
// outside the reduction range (never produced by the codec's activations) take sinf.
// Accuracy <= 3.5 ulp (tests/test_gpu_kernels.py::test_snake measures it against fp64).
// Round 3: q = rint(x / pi) as (t + 1.5 * 2^23) - 1.5 * 2^23 (round-to-nearest-even, exact for |t| < 2^22, so
// equal to rintf), whose low mantissa bit is q's parity; the odd-q sign is applied to the RESULT by an xor
// instead of negating d first: fma(s, u * (-d), -d) = -fma(s, u * d, d) exactly (s = d * d), so the value is
// bit-identical to the previous rintf / cvt / and / cmp / negate / select form, in 5 fewer instructions.
constexpr float BC_RINT_MAGIC = 12582912.0f;  // 1.5 * 2^23
__device__ __forceinline__ float bc_sin(float x) {
  if (!(fabsf(x) < 39000.0f)) return sinf(x);
  const float qm = x * 0.318309886183790671538f + BC_RINT_MAGIC;  // (two roundings: no fma contraction)
  const float q = qm - BC_RINT_MAGIC;
  float d = fmaf(q, -3.140625f, x);
  d = fmaf(q, -0.0009670257568359375f, d);
  d = fmaf(q, -6.2771141529083251953e-07f, d);
  d = fmaf(q, -1.2154201256553420762e-10f, d);
  const float s = d * d;
  float u = 2.6083159809786593541503e-06f;
  u = fmaf(u, s, -0.0001981069071916863322258f);
  u = fmaf(u, s, 0.00833307858556509017944336f);
  u = fmaf(u, s, -0.166666597127914428710938f);
  const float r = fmaf(s, u * d, d);
  return __uint_as_float(__float_as_uint(r) ^ (__float_as_uint(qm) << 31));
}

// SnakeBeta (vq/activations.py:107-118):  x + (1/(exp(b)+1e-9)) * sin(x*exp(a))^2.
// alpha_exp = exp(a) and inv_beta = 1/(exp(b)+1e-9) are precomputed per channel on the host with
// the same torch CPU expressions the reference evaluates, so only the per-element part runs here:
// t = x*alpha; s = sin(t); y = x + inv_beta*(s*s)   (pow(s,2) == s*s in torch).
__device__ __forceinline__ float snake(float x, float alpha_exp, float inv_beta) {
  const float s = bc_sin(x * alpha_exp);
  return x + inv_beta * (s * s);
}

// The same two functions on pairs, written so the fp32 arithmetic issues as packed v_pk_fma_f32 /
// v_pk_mul_f32 / v_pk_add_f32 (two lanes' worth of work per instruction: the epilogues that apply
// a Snake to every output element are VALU-heavy).  Each component rounds exactly as bc_sin /
// snake above (same operations, same order), so the results are bit-identical to them.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 splat2(float v) { return (f32x2){v, v}; }
__device__ __forceinline__ f32x2 bc_sin_pk(f32x2 x) {
  const f32x2 qm = x * splat2(0.318309886183790671538f) + splat2(BC_RINT_MAGIC);
  const f32x2 q = qm - splat2(BC_RINT_MAGIC);
  f32x2 d = __builtin_elementwise_fma(q, splat2(-3.140625f), x);
  d = __builtin_elementwise_fma(q, splat2(-0.0009670257568359375f), d);
  d = __builtin_elementwise_fma(q, splat2(-6.2771141529083251953e-07f), d);
  d = __builtin_elementwise_fma(q, splat2(-1.2154201256553420762e-10f), d);
  const f32x2 s = d * d;
  f32x2 u = splat2(2.6083159809786593541503e-06f);
  u = __builtin_elementwise_fma(u, s, splat2(-0.0001981069071916863322258f));
  u = __builtin_elementwise_fma(u, s, splat2(0.00833307858556509017944336f));
  u = __builtin_elementwise_fma(u, s, splat2(-0.166666597127914428710938f));
  f32x2 r = __builtin_elementwise_fma(s, u * d, d);
  r.x = __uint_as_float(__float_as_uint(r.x) ^ (__float_as_uint(qm.x) << 31));
  r.y = __uint_as_float(__float_as_uint(r.y) ^ (__float_as_uint(qm.y) << 31));
  if (!(fabsf(x.x) < 39000.0f)) r.x = sinf(x.x);
  if (!(fabsf(x.y) < 39000.0f)) r.y = sinf(x.y);
  return r;
}
__device__ __forceinline__ f32x2 snake_pk(f32x2 x, f32x2 alpha_exp, f32x2 inv_beta) {
  const f32x2 s = bc_sin_pk(x * alpha_exp);
  return x + inv_beta * (s * s);
}

// Bijective XCD-aware remap of a 1-D workgroup id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): workgroups that the dispatcher deals to the same XCD (ids b, b+8, b+16, ...) receive
// consecutive logical ids, so neighbouring tiles that share an input panel share one L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
#ifdef BC_NO_XCD_REMAP  // experiment builds only (BIGCODEC_NO_XCD_REMAP=1): the dispatcher's own order
  return orig;
#endif
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8, loc = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Workgroup barrier for LDS hand-offs that leaves outstanding global loads in flight: the compiler
// drains vmcnt in front of __syncthreads(), which would also wait for prefetches meant to land
// later.  LDS writes are drained (lgkmcnt), the "memory" clobber keeps the compiler from moving
// memory accesses across it; LDS-DMA that must have landed is waited for explicitly (vmcnt).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float sigmoidf_ref(float x) { return 1.0f / (1.0f + expf(-x)); }

// splitmix64 finalizer (SURVEY.md §8(d) synthetic input spec).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace bc
