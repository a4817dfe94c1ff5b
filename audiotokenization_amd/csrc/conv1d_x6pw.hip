// x6 pointwise conv (K = 1) with a DOUBLE-BUFFERED input tile: the ResidualUnit k1 convs at C = 192 / 384 / 768
// (vq/module.py:83-89: conv1(snake2(h)) + x, the next unit's Snake as a dual output) in the exact 3 x bf16 arithmetic of
// conv1d_x6_kernel.h.
//
// Why: on the 16-wave 192 x 256 tile a pointwise conv has one K-step per 32-channel chunk, and the chunk's three B planes
// (48 KiB at 256 columns) leave no LDS for a second B buffer next to the double-buffered A block (2 x 36 KiB): every
// chunk ends with a barrier, the split + store of the next chunk by all 16 waves with no MFMA beside it, a wait and a
// second barrier.  Here the tile is 192 x 192 (16 waves of 48 x 48, 3 x 3 MFMA tiles each): the B planes of a chunk are
// 36 KiB, so A and B are both double-buffered (144 KiB) and a chunk costs ONE barrier; each wave stores its share of
// chunk c + 1's planes between its first and its other m-tiles of chunk c, so the staging runs beside the other waves'
// MFMAs, and issues chunk c + 1's A copy and chunk c + 2's 16-byte loads right after.  Per K32 unit a wave reads 9 A + 9 B fragments for 54
// MFMAs (the 16-wave tile: 18 + 6 for 72).
//
// Arithmetic: the same B planes (split2 of the same fp32 values), the same A planes (the cfg-122 packing: 12 m-tiles of
// 16 rows per 192-row group), the same chunk order and six-MFMA chain per output as conv1d_x6_kernel<..., P = 3>, the
// shared epilogue: outputs bit-identical to the 16-wave tile (tests/test_gpu_kernels.py::test_x6pw_bit_identical).
#include "bc_common.h"
#include "bc_internal.h"
#include "conv_epilogue.h"
#include "x6_common.h"

namespace bc {

constexpr int PWD_MT = 3, PWD_NT = 3, PWD_WM = 4, PWD_WN = 4, PWD_NW = PWD_WM * PWD_WN;
constexpr int PWD_BM = 16 * PWD_MT * PWD_WM;  // 192
constexpr int PWD_BN = 16 * PWD_NT * PWD_WN;  // 192
constexpr int PWD_QA = PWD_WM * PWD_MT;       // 12 m-tiles per row group (the cfg-122 packing)
constexpr int PWD_APIECES = 3 * PWD_QA;       // 36 KiB of A per chunk
constexpr int PWD_BPLANE = PWD_BN * 64;       // 12 KiB per B plane
constexpr int PWD_LDS = 2 * 3 * PWD_BPLANE + 2 * PWD_APIECES * 1024;  // 144 KiB
constexpr int PWD_NPQ = 16 * (PWD_BN / 4);    // (channel pair, column quad) items of a chunk: 768 (one per thread)

__global__ void __launch_bounds__(1024, 1) conv1d_x6pw_kernel(ConvArgs a) {
  constexpr int MT = PWD_MT, NT = PWD_NT, WM = PWD_WM, NW = PWD_NW;
  typedef bf16x8_t frag_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_pwd[];
  unsigned char* Bs = smem_pwd;                      // [2][3 planes][192 columns][64 B] (swizzled 16-B groups)
  unsigned char* As = smem_pwd + 2 * 3 * PWD_BPLANE;  // [2][3 planes][12 m-tiles][1 KiB]
  auto bgrp = [](int col, int g) __attribute__((always_inline)) { return col * 64 + 16 * (g ^ ((col >> 1) & 3)); };

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int mt_idx = wg % a.ntm;
  const int rest = wg / a.ntm;
  const int nt_idx = rest % a.ntn;
  const int b = rest / a.ntn;
  const int m0 = mt_idx * PWD_BM;
  const int n0 = nt_idx * PWD_BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM;
  const int wn = wave / WM;

  const unsigned long long xb_u = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned xb_lo = __builtin_amdgcn_readfirstlane((unsigned)xb_u);
  const unsigned xb_hi = __builtin_amdgcn_readfirstlane((unsigned)(xb_u >> 32));
  const int xbytes = __builtin_amdgcn_readfirstlane(a.Cin * a.Tin * 4);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long long)xb_hi << 32) | xb_lo), 0, xbytes, 0x00020000);
  const int nch = a.nchunks;
  const unsigned char* wblk = reinterpret_cast<const unsigned char*>(a.w) + (long long)mt_idx * nch * (PWD_APIECES * 1024);

  // A block of chunk c (36 pieces over the 16 waves) into A buffer c & 1: EXACTLY three copies per wave (waves 4-15
  // repeat their second piece as the third: the same bytes to the same LDS address), so the compiler's counted waits
  // for the staging registers see a static number of younger vector-memory ops (a per-wave trip count made it drain
  // vmcnt(0), the fresh copy included)
  auto issue_a = [&](int c) __attribute__((always_inline)) {
    const unsigned char* src = wblk + (long long)c * (PWD_APIECES * 1024);
    unsigned char* dst = As + (c & 1) * (PWD_APIECES * 1024);
    if (!BC_DOK(mt_idx < a.ntm && c < nch)) return;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int q = wave + NW * k < PWD_APIECES ? wave + NW * k : wave + NW;
      __builtin_amdgcn_global_load_lds((const void*)(src + q * 1024 + lane * 16), (lds_void_t)(dst + q * 1024), 16, 0,
                                       0);
    }
  };
  // B staging: thread t < 768 holds channel pair t % 16 and column quad t / 16 of a chunk (two 16-byte loads; columns
  // n0 + 4q .. + 3, all inside or all past Tin since Tin % 4 == 0: past it the buffer load reads 0)
  const bool stg = tid < PWD_NPQ;
  const int sp = tid & 15, sq = tid >> 4;
  floatx4 s0, s1;
  auto load_b = [&](int c) __attribute__((always_inline)) {
    const int c0 = c * X6_BKC + 2 * sp;
    const int t = n0 + 4 * sq;
    const bool ok = stg && t < a.Tin;
    const unsigned o0 = (ok && c0 < a.Cin) ? (unsigned)((c0 * a.Tin + t) * 4) : 0x80000000u;
    const unsigned o1 = (ok && c0 + 1 < a.Cin) ? (unsigned)(((c0 + 1) * a.Tin + t) * 4) : 0x80000000u;
    s0 = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o0, 0, 0));
    s1 = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o1, 0, 0));
  };
  auto store_b = [&](int c) __attribute__((always_inline)) {
    // every wave (the four non-staging ones too) consumes its loads here: without this the compiler carries the skipped
    // waves' loads past the A copy and drains vmcnt to zero before the next load_b reuses the registers
    asm volatile("" ::"v"(s0), "v"(s1));
    if (!stg) return;
    unsigned char* Bt = Bs + (c & 1) * (3 * PWD_BPLANE);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unsigned h, m, l;
      split2(s0[j], s1[j], h, m, l);
      unsigned char* p = Bt + bgrp(4 * sq + j, sp >> 2) + (sp & 3) * 4;
      *reinterpret_cast<unsigned*>(p) = h;
      *reinterpret_cast<unsigned*>(p + PWD_BPLANE) = m;
      *reinterpret_cast<unsigned*>(p + 2 * PWD_BPLANE) = l;
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int col_lane = wn * NT * 16 + (lane & 15);
  auto mtile = [&](int c, int i, const frag_t (&bf)[NT][3]) __attribute__((always_inline)) {
    const unsigned char* Aq = As + (c & 1) * (PWD_APIECES * 1024) + (wm * MT + i) * 1024 + lane * 16;
    const frag_t a0 = *reinterpret_cast<const frag_t*>(Aq);
    const frag_t a1 = *reinterpret_cast<const frag_t*>(Aq + PWD_QA * 1024);
    const frag_t a2 = *reinterpret_cast<const frag_t*>(Aq + 2 * PWD_QA * 1024);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      // conv1d_x6_kernel<..., P = 3>'s chain, in its order (operands swapped: input as A)
      floatx4 t = acc[i][j];
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a2, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a1, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][2], a0, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a1, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a0, t, 0, 0, 0);
      t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a0, t, 0, 0, 0);
      acc[i][j] = t;
    }
  };

  // prologue: A(0) and the planes of chunk 0 in buffer 0, chunk 1's loads in flight
  issue_a(0);
  dma_issue_order();
  load_b(0);
  store_b(0);
  if (nch > 1) load_b(1);
  if (nch > 1) wait_vmcnt<2>();  // A(0) landed (chunk 1's two loads may stay in flight)
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  for (int c = 0; c < nch; ++c) {
    const unsigned char* Bcol = Bs + (c & 1) * (3 * PWD_BPLANE) + bgrp(col_lane, lane >> 4);
    frag_t bf[NT][3];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) bf[j][p] = *reinterpret_cast<const frag_t*>(Bcol + j * 16 * 64 + p * PWD_BPLANE);
    mtile(c, 0, bf);
    // chunk c + 1's planes (loaded a whole chunk ago) and A block go into the buffers chunk c - 1 used (freed by its
    // barrier); the A copy is issued AFTER the store, so the compiler's wait for the staging registers (it drains
    // vmcnt to zero for them whatever LDS-DMA follows) never waits for the fresh copy
    if (c + 1 < nch) {
      store_b(c + 1);
      issue_a(c + 1);
      dma_issue_order();
      if (c + 2 < nch) load_b(c + 2);
    }
#pragma unroll
    for (int i = 1; i < MT; ++i) mtile(c, i, bf);
    // A(c + 1) must have landed; chunk c + 2's two loads (issued after it) may stay in flight
    if (c + 2 < nch) wait_vmcnt<2>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();  // chunk c + 1's planes and A block visible; every wave done with buffers c & 1
  }

  conv_epilogue<MT, NT>(a, acc, b, m0 + wm * MT * 16, n0 + wn * NT * 16, lane);
}

bool x6pw_fits(const ConvArgs& a) {
  return a.K == 1 && a.s == 1 && a.d == 1 && a.pl == 0 && a.ps == 0 && a.Cout % PWD_BM == 0 && a.Tin == a.Nout &&
         a.Tin % 4 == 0 && a.xbs % 4 == 0 && ((unsigned long long)a.x & 15) == 0;
}

// BC_X6_PWDB=0 keeps the pointwise x6 convs on the 16-wave tile (A/B timing)
bool x6pw_on() {
  static const bool v = [] {
    const char* e = getenv("BC_X6_PWDB");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// a: a pointwise x6 conv as x6_launch prepared it, weights packed for cfg 122 (192-row groups)
int x6pw_launch(ConvArgs& a, int B, hipStream_t st) {
  if (!x6pw_fits(a)) return BC_ERR_UNSUPPORTED;
  a.ntm = a.Cout / PWD_BM;
  a.ntn = (a.Nout + PWD_BN - 1) / PWD_BN;
  a.nchunks = (a.Cin + X6_BKC - 1) / X6_BKC;
  a.win = PWD_BN;
  a.bpitch = 64;
  a.bstage = PWD_BPLANE;
  const long long nwg = (long long)a.ntm * a.ntn * B;
  if (nwg <= 0) return BC_OK;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  if ((long long)a.Cin * a.Tin * 4 > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  a.nwg = (int)nwg;
  a.wsc = nullptr;
  hipLaunchKernelGGL(conv1d_x6pw_kernel, dim3(a.nwg), dim3(1024), PWD_LDS, st, a);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

}  // namespace bc

BC_DEBUG_EXPORT(conv1d_x6pw)
