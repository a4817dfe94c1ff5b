// Minimal repro for the resunit_rr note: a v_mfma_f32_16x16x16_f16 whose SrcC is the vDST of
// the v_mfma_f32_16x16x32_f16 just before it (the chain resunit_rr.hip avoids).  Compile to ISA and count
// the wait states hipcc puts between the two:
//   hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S tools/isa_repro/mfma_chain.hip -o /tmp/chain.s
// tools/isa_repro/check_chain.py reads the result.
#include <hip/hip_runtime.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void chain_32_then_16(const f16x8* a, const f16x8* b, const f16x4* c, const f16x4* d, f32x4* out) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[l], b[l], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[l + 64], b[l + 64], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(c[l], d[l], acc, 0, 0, 0);  // SrcC = the 16x16x32's vDST
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(c[l + 64], d[l + 64], acc, 0, 0, 0);
  out[l] = acc;
}

__global__ void chain_16_then_32(const f16x8* a, const f16x8* b, const f16x4* c, const f16x4* d, f32x4* out) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x16f16(c[l], d[l], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[l], b[l], acc, 0, 0, 0);  // SrcC = the 16x16x16's vDST
  out[l] = acc;
}

__global__ void chain_32_then_32(const f16x8* a, const f16x8* b, f32x4* out) {
  const int l = threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[l], b[l], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[l + 64], b[l + 64], acc, 0, 0, 0);
  out[l] = acc;
}

// ---- hardware check: the chain as hipcc emits it (no wait states) vs the same chain with a gap of GAP wait
// states (s_nop GAP-1; GAP = 0: back to back) and vs a fully padded reference (16 wait states).  ORDER 0: 16x16x32
// then 16x16x16 reading its vDST as SrcC; ORDER 1: 16x16x16 then 16x16x32; ORDER 2: 16x16x32 twice.
// Each wave computes its own random operands.
template <int ORDER, int GAP>
__global__ void chain_probe(const f16x8* a, const f16x8* b, const f16x4* c, const f16x4* d, f32x4* out) {
  const int g = blockIdx.x * 64 + threadIdx.x;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const f16x8 av = a[g], bv = b[g], a2 = a[g ^ 1], b2 = b[g ^ 1];
  const f16x4 cv = c[g], dv = d[g];
  __builtin_amdgcn_sched_barrier(0);
  if (ORDER == 1) acc = __builtin_amdgcn_mfma_f32_16x16x16f16(cv, dv, acc, 0, 0, 0);
  else acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bv, acc, 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  if (GAP > 0) asm volatile("s_nop %0" ::"n"(GAP > 8 ? 7 : GAP - 1));
  if (GAP > 8) asm volatile("s_nop 7" ::);
  __builtin_amdgcn_sched_barrier(0);
  if (ORDER == 0) acc = __builtin_amdgcn_mfma_f32_16x16x16f16(cv, dv, acc, 0, 0, 0);
  else acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ORDER == 2 ? a2 : av, ORDER == 2 ? b2 : bv, acc, 0, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  out[g] = acc;
}

#define CHAIN_CASE(O, G) \
  case G: hipLaunchKernelGGL((chain_probe<O, G>), dim3(waves), dim3(64), 0, 0, A, Bp, Cp, Dp, O_); break;
#define CHAIN_ORDER(O)                                                                                          \
  case O:                                                                                                       \
    switch (gap) { CHAIN_CASE(O, 0) CHAIN_CASE(O, 1) CHAIN_CASE(O, 2) CHAIN_CASE(O, 3) CHAIN_CASE(O, 4)         \
                   CHAIN_CASE(O, 5) CHAIN_CASE(O, 6) CHAIN_CASE(O, 8) CHAIN_CASE(O, 16) default: return 2; }  \
    break;

// order 0/1/2, gap in {0..6, 8, 16}
extern "C" int mfma_chain_probe(const void* a, const void* b, const void* c, const void* d, void* out, int waves,
                                int order, int gap) {
  const f16x8 *A = (const f16x8*)a, *Bp = (const f16x8*)b;
  const f16x4 *Cp = (const f16x4*)c, *Dp = (const f16x4*)d;
  f32x4* O_ = (f32x4*)out;
  switch (order) { CHAIN_ORDER(0) CHAIN_ORDER(1) CHAIN_ORDER(2) default: return 2; }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
