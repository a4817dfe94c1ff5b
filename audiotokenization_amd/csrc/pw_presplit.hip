// Pointwise GEMM with a pre-split B operand: the ResLSTM input projection gx = W_ih x + b over T*B columns
// (vq/module.py:143-167 -> nn.LSTM's input-hidden product; Cin = H = 1536, Cout = 4H = 6144 in the default
// model), h3 operands.
//
// On the 16-wave 192 x 256 tile (cfg 322) every m-tile workgroup re-stages the same B chunk: 32 of them per
// column tile here, each loading 32 channels x 256 columns of fp32, taking the block maximum, splitting into two
// fp16 planes and storing them to LDS, between two barriers and with no MFMA to overlap (one chunk = one K-step
// for a pointwise conv).  Measured: 6.7k cycles per chunk-step against 2.3k of MFMA.  Here:
//   presplit_b_kernel  one pass over x: per 256-column tile and 32-channel chunk the block scale exactly as the
//                      GEMM's staging computes it (h3_scale_from_bits of the block maximum, out-of-range columns
//                      zero; the running minimum over the tile's chunks so far), and the two fp16 planes of
//                      x * scale in the GEMM's LDS image ([col][64 B], 16-B channel groups XOR-swizzled by
//                      (col >> 1) & 3), so the GEMM copies them with LDS-DMA like the weights;
//   pw_presplit_kernel the 16-wave tile's main loop with B by LDS-DMA (double-buffered A and B, one barrier per
//                      chunk, no staging VALU), the same MFMA chain per output and the same exact power-of-two
//                      accumulator rescale when the scale decreases, the shared h3 epilogue.
// Same blocks, same scales, same products in the same order: bit-identical to conv1d_x6_kernel on cfg 322
// (tests/test_gpu_kernels.py::test_lstm_projection_presplit_bit_identical).
#include "bc_common.h"
#include "bc_internal.h"
#include "conv_epilogue.h"
#include "x6_common.h"

namespace bc {

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

constexpr int PS_BN = 256;             // columns per tile: the 16-wave tile's BN (the same staged blocks)
constexpr int PS_PLANE = PS_BN * 64;   // bytes of one fp16 plane of a chunk (32 channels per column)
constexpr int PS_MT = 6, PS_NT = 2, PS_WM = 2, PS_WN = 8;
constexpr int PS_QA = PS_WM * PS_MT;   // 12 m-tiles of 16 rows
constexpr int PS_APIECES = 2 * PS_QA;  // 1-KiB pieces of a chunk's A block (2 planes)
constexpr int PS_BPIECES = 2 * PS_PLANE / 1024;  // 32 pieces of a chunk's B block
constexpr int PS_BBUF = 3;             // B buffers: chunk c + 2's planes are in flight while chunk c computes
constexpr int PS_LDS = PS_BBUF * 2 * PS_PLANE + 2 * PS_APIECES * 1024;  // 144 KiB

// One 256-thread workgroup per 256-column tile: wave w holds channels 8w .. 8w + 7 of each chunk, lane l the
// columns 4l .. 4l + 3 (16-byte loads, 1 KiB per channel row per wave).
__global__ void __launch_bounds__(256) presplit_b_kernel(const float* __restrict__ x, unsigned char* __restrict__ planes,
                                                         float* __restrict__ scales, int Cin, int N, int nch) {
  const int j = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = j * PS_BN + 4 * lane;
  __shared__ unsigned wmax[4];
  float xs = 1.f;
  // chunk c + 1's rows are loaded while chunk c is reduced and split (two register sets): the per-chunk work is the
  // same, the loads of the next chunk no longer wait behind this chunk's two barriers
  auto load = [&](int c, float (&v)[8][4]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ch = c * X6_BKC + 8 * w + k;
      const float* row = x + (long long)ch * N;
      if (ch < Cin && n + 3 < N && (N & 3) == 0) {  // 16-byte aligned rows
        const floatx4 q = *reinterpret_cast<const floatx4*>(row + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[k][r] = q[r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[k][r] = (ch < Cin && n + r < N) ? row[n + r] : 0.f;
      }
    }
  };
  auto body = [&](int c, const float (&v)[8][4]) {
    unsigned m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const unsigned u = __float_as_uint(fabsf(v[k][r]));
        m = m > u ? m : u;
      }
    m = wave_max_u32(m);
    if (lane == 0) wmax[w] = m;
    __syncthreads();
    unsigned mm = wmax[0];
#pragma unroll
    for (int q = 1; q < 4; ++q) mm = mm > wmax[q] ? mm : wmax[q];
    const float s = h3_scale_from_bits(__builtin_amdgcn_readfirstlane(mm));
    xs = c == 0 ? s : (s < xs ? s : xs);  // the GEMM's staging: chunk 0's scale, then the running minimum
    __syncthreads();                      // wmax is rewritten by the next chunk
    if (tid == 0) scales[(long long)j * nch + c] = xs;
    unsigned char* pb = planes + ((long long)j * nch + c) * (2 * PS_PLANE);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = 4 * lane + r;
      unsigned h[4], l[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) split2_h(v[2 * k][r] * xs, v[2 * k + 1][r] * xs, h[k], l[k]);
      const int off = col * 64 + 16 * (w ^ ((col >> 1) & 3));
      *reinterpret_cast<u32x4_t*>(pb + off) = (u32x4_t){h[0], h[1], h[2], h[3]};
      *reinterpret_cast<u32x4_t*>(pb + PS_PLANE + off) = (u32x4_t){l[0], l[1], l[2], l[3]};
    }
  };
  float va[8][4], vb[8][4];
  if (nch > 0) load(0, va);
  for (int c = 0; c < nch; c += 2) {
    if (c + 1 < nch) load(c + 1, vb);
    body(c, va);
    if (c + 1 < nch) {
      if (c + 2 < nch) load(c + 2, va);
      body(c + 1, vb);
    }
  }
}

__global__ void __launch_bounds__(1024, 1) pw_presplit_kernel(ConvArgs a, const unsigned char* __restrict__ planes,
                                                              const float* __restrict__ scales) {
  constexpr int MT = PS_MT, NT = PS_NT, WM = PS_WM, NW = PS_WM * PS_WN;
  typedef f16x8_t frag_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_ps[];
  unsigned char* Bs = smem_ps;                           // [3][2 planes][PS_PLANE]
  unsigned char* As = smem_ps + PS_BBUF * 2 * PS_PLANE;  // [2][2 planes][QA][1 KiB]

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int mt_idx = wg % a.ntm;
  const int nt_idx = wg / a.ntm;
  const int m0 = mt_idx * 16 * MT * WM;
  const int n0 = nt_idx * PS_BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int nch = a.nchunks;

  const unsigned char* wblk = reinterpret_cast<const unsigned char*>(a.w) + (long long)mt_idx * nch * (PS_APIECES * 1024);
  const unsigned char* bblk = planes + (long long)nt_idx * nch * (2 * PS_PLANE);
  const float* sblk = scales + (long long)nt_idx * nch;
  // chunk c's A block (24 pieces; A buffer c & 1) and B block (32 pieces, exactly 2 per wave; B buffer c % 3),
  // spread over the 16 waves
  static_assert(PS_BPIECES == 2 * NW, "two B pieces per wave (the counted wait below)");
  auto issue_a = [&](int c) {
    const unsigned char* sa = wblk + (long long)c * (PS_APIECES * 1024);
    unsigned char* da = As + (c & 1) * (PS_APIECES * 1024);
    for (int q = wave; q < PS_APIECES; q += NW)
      __builtin_amdgcn_global_load_lds((const void*)(sa + q * 1024 + lane * 16), (lds_void_t)(da + q * 1024), 16, 0, 0);
  };
  auto issue_b = [&](int c) {
    const unsigned char* sb = bblk + (long long)c * (2 * PS_PLANE);
    unsigned char* db = Bs + (c % PS_BBUF) * (2 * PS_PLANE);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = wave + k * NW;
      __builtin_amdgcn_global_load_lds((const void*)(sb + q * 1024 + lane * 16), (lds_void_t)(db + q * 1024), 16, 0, 0);
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int col_lane = wn * NT * 16 + (lane & 15);
  const int bgo = col_lane * 64 + 16 * ((lane >> 4) ^ ((col_lane >> 1) & 3));  // conv1d_x6_kernel's bgrp
  // one chunk: this wave's MT x NT tiles, A fragments one m-tile ahead (conv1d_x6_kernel's compute, h3)
  auto compute = [&](int c) {
    const unsigned char* Ab = As + (c & 1) * (PS_APIECES * 1024);
    const unsigned char* Bcol = Bs + (c % PS_BBUF) * (2 * PS_PLANE) + bgo;
    frag_t bf[NT][2];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) bf[j][p] = *reinterpret_cast<const frag_t*>(Bcol + j * 16 * 64 + p * PS_PLANE);
    frag_t af[2][2];
    auto load_a = [&](int i, frag_t (&d)[2]) {
      const unsigned char* Aq = Ab + (wm * MT + i) * 1024 + lane * 16;
#pragma unroll
      for (int p = 0; p < 2; ++p) d[p] = *reinterpret_cast<const frag_t*>(Aq + p * PS_QA * 1024);
    };
    load_a(0, af[0]);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      const frag_t a0 = af[i & 1][0], a1 = af[i & 1][1];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if (j == 1 && i + 1 < MT) {
          __builtin_amdgcn_sched_barrier(0);
          load_a(i + 1, af[(i + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
        }
        floatx4 t = acc[i][j];
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][1], a0, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][0], a1, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][0], a0, t, 0, 0, 0);
        acc[i][j] = t;
      }
    }
  };

  // issue order per wave: B(0), A(0), B(1) | step c: A(c + 1), B(c + 2), compute, counted wait, barrier.  vmcnt
  // retires in issue order, so at the end of step c a wait for all but this wave's 2 youngest pieces (B(c + 2))
  // retires A(c + 1) and B(c + 1); the barrier then publishes every wave's pieces and frees A buffer c & 1 and B
  // buffer c % 3 (rewritten by A(c + 2) / B(c + 3), issued in steps c + 1 / c + 1).
  issue_b(0);
  issue_a(0);
  dma_issue_order();
  if (nch > 1) issue_b(1);
  float xs = sblk[0];
  if (nch > 1) wait_vmcnt<2>();
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) issue_a(c + 1);
    dma_issue_order();
    if (c + 2 < nch) issue_b(c + 2);
    dma_issue_order();
    compute(c);
    if (c + 1 < nch) {  // chunk c + 1 was split at the running-minimum scale: follow it exactly (powers of two)
      const float sn = sblk[c + 1];
      if (sn < xs) {
        const float r = sn / xs;
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] *= r;
        xs = sn;
      }
    }
    if (c + 2 < nch)
      wait_vmcnt<2>();  // this wave's pieces of A(c + 1) and B(c + 1) have landed; B(c + 2) may stay in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
  }
  conv_epilogue<MT, NT, true>(a, acc, 0, m0 + wm * MT * 16, n0 + wn * NT * 16, lane, 1.f / xs);
}

// ------------------------------------------------------------------------------------------------
// x6 (P = 3): the same idea without block scales (the 3 x bf16 split is exact per element).  Three planes of a
// 256-column chunk are 48 KiB, so the 192-row GEMM's A + B double buffers (2 x 36 + 2 x 48 KiB) would exceed the
// 160 KiB LDS: the x6 GEMM tile is 128 rows x 256 columns (16 waves of 64 x 32, 4 x 2 MFMA tiles each), A and B
// double-buffered (2 x 24 + 2 x 48 = 144 KiB).  A comes from the weights packed for cfg 122 (192-row groups): its
// 1-KiB pieces are per (16-row m-tile, plane, chunk), so any 16-row-aligned tile gathers them piece by piece.
// Per output the same chunk order and the same six-MFMA chain as conv1d_x6_kernel<..., P = 3>: bit-identical to
// the cfg-122 x6 launch (tests/test_gpu_kernels.py::test_lstm_projection_presplit_bit_identical[x6]).
constexpr int PX_MT = 4, PX_NT = 2, PX_WM = 2, PX_WN = 8;
constexpr int PX_BM = 16 * PX_MT * PX_WM;  // 128
constexpr int PX_QA = PX_WM * PX_MT;       // 8 m-tiles
constexpr int PX_APIECES = 3 * PX_QA;      // 24 pieces of a chunk's A block
constexpr int PX_BPIECES = 3 * PS_PLANE / 1024;  // 48 pieces of a chunk's B block (3 per wave)
constexpr int PX_LDS = 2 * 3 * PS_PLANE + 2 * PX_APIECES * 1024;  // 144 KiB
constexpr int P122_QA = 12;                // m-tiles per 192-row group of the cfg-122 packing

__global__ void __launch_bounds__(256) presplit_b_x6_kernel(const float* __restrict__ x, unsigned char* __restrict__ planes,
                                                            int Cin, int N, int nch) {
  const int j = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = j * PS_BN + 4 * lane;
  auto load = [&](int c, float (&v)[8][4]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int ch = c * X6_BKC + 8 * w + k;
      const float* row = x + (long long)ch * N;
      if (ch < Cin && n + 3 < N && (N & 3) == 0) {
        const floatx4 q = *reinterpret_cast<const floatx4*>(row + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[k][r] = q[r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[k][r] = (ch < Cin && n + r < N) ? row[n + r] : 0.f;
      }
    }
  };
  auto body = [&](int c, const float (&v)[8][4]) {
    unsigned char* pb = planes + ((long long)j * nch + c) * (3 * PS_PLANE);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = 4 * lane + r;
      unsigned h[4], m[4], l[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) split2(v[2 * k][r], v[2 * k + 1][r], h[k], m[k], l[k]);
      const int off = col * 64 + 16 * (w ^ ((col >> 1) & 3));
      *reinterpret_cast<u32x4_t*>(pb + off) = (u32x4_t){h[0], h[1], h[2], h[3]};
      *reinterpret_cast<u32x4_t*>(pb + PS_PLANE + off) = (u32x4_t){m[0], m[1], m[2], m[3]};
      *reinterpret_cast<u32x4_t*>(pb + 2 * PS_PLANE + off) = (u32x4_t){l[0], l[1], l[2], l[3]};
    }
  };
  float va[8][4], vb[8][4];
  if (nch > 0) load(0, va);
  for (int c = 0; c < nch; c += 2) {
    if (c + 1 < nch) load(c + 1, vb);
    body(c, va);
    if (c + 1 < nch) {
      if (c + 2 < nch) load(c + 2, va);
      body(c + 1, vb);
    }
  }
}

__global__ void __launch_bounds__(1024, 1) pw_presplit_x6_kernel(ConvArgs a, const unsigned char* __restrict__ planes) {
  constexpr int MT = PX_MT, NT = PX_NT, WM = PX_WM, NW = PX_WM * PX_WN;
  typedef bf16x8_t frag_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_px[];
  unsigned char* Bs = smem_px;                        // [2][3 planes][PS_PLANE]
  unsigned char* As = smem_px + 2 * 3 * PS_PLANE;     // [2][3 planes][QA][1 KiB]

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int mt_idx = wg % a.ntm;
  const int nt_idx = wg / a.ntm;
  const int m0 = mt_idx * PX_BM;
  const int n0 = nt_idx * PS_BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int nch = a.nchunks;

  const unsigned char* wbase = reinterpret_cast<const unsigned char*>(a.w);
  const unsigned char* bblk = planes + (long long)nt_idx * nch * (3 * PS_PLANE);
  // A piece q = plane * QA + local m-tile: m-tile g = m0 / 16 + local of the cfg-122 packing
  // [group g / 12][chunk][plane][g % 12][1 KiB]
  auto issue_a = [&](int c) {
    unsigned char* da = As + (c & 1) * (PX_APIECES * 1024);
    for (int q = wave; q < PX_APIECES; q += NW) {
      const int p = q / PX_QA, g = m0 / 16 + q % PX_QA;
      const unsigned char* src =
          wbase + ((((long long)(g / P122_QA) * nch + c) * 3 + p) * P122_QA + g % P122_QA) * 1024;
      __builtin_amdgcn_global_load_lds((const void*)(src + lane * 16), (lds_void_t)(da + q * 1024), 16, 0, 0);
    }
  };
  auto issue_b = [&](int c) {
    const unsigned char* sb = bblk + (long long)c * (3 * PS_PLANE);
    unsigned char* db = Bs + (c & 1) * (3 * PS_PLANE);
#pragma unroll
    for (int k = 0; k < PX_BPIECES / NW; ++k) {
      const int q = wave + k * NW;
      __builtin_amdgcn_global_load_lds((const void*)(sb + q * 1024 + lane * 16), (lds_void_t)(db + q * 1024), 16, 0, 0);
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int col_lane = wn * NT * 16 + (lane & 15);
  const int bgo = col_lane * 64 + 16 * ((lane >> 4) ^ ((col_lane >> 1) & 3));  // conv1d_x6_kernel's bgrp
  auto compute = [&](int c) {
    const unsigned char* Ab = As + (c & 1) * (PX_APIECES * 1024);
    const unsigned char* Bcol = Bs + (c & 1) * (3 * PS_PLANE) + bgo;
    frag_t bf[NT][3];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) bf[j][p] = *reinterpret_cast<const frag_t*>(Bcol + j * 16 * 64 + p * PS_PLANE);
    frag_t af[2][3];
    auto load_a = [&](int i, frag_t (&d)[3]) {
      const unsigned char* Aq = Ab + (wm * MT + i) * 1024 + lane * 16;
#pragma unroll
      for (int p = 0; p < 3; ++p) d[p] = *reinterpret_cast<const frag_t*>(Aq + p * PX_QA * 1024);
    };
    load_a(0, af[0]);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      const frag_t a0 = af[i & 1][0], a1 = af[i & 1][1], a2 = af[i & 1][2];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if (j == 1 && i + 1 < MT) {
          __builtin_amdgcn_sched_barrier(0);
          load_a(i + 1, af[(i + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);
        }
        // conv1d_x6_kernel<..., P = 3>'s chain, in its order
        floatx4 t = acc[i][j];
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a2, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a1, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][2], a0, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a1, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a0, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a0, t, 0, 0, 0);
        acc[i][j] = t;
      }
    }
  };

  // step c: A(c + 1) and B(c + 1) into the buffers chunk c - 1 used (freed by step c - 1's barrier), compute chunk
  // c, wait for this wave's copies, barrier (every wave's copies have landed, every wave is done with buffer c & 1)
  issue_a(0);
  dma_issue_order();
  issue_b(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) {
      issue_a(c + 1);
      dma_issue_order();
      issue_b(c + 1);
      dma_issue_order();
    }
    compute(c);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
  }
  conv_epilogue<MT, NT>(a, acc, 0, m0 + wm * MT * 16, n0 + wn * NT * 16, lane);
}

long long pw_presplit_bytes(int Cin, long long N) {
  // the larger of the two layouts: x6's three planes (no scales) >= h3's two planes + one scale per chunk
  const long long ntn = (N + PS_BN - 1) / PS_BN, nch = (Cin + X6_BKC - 1) / X6_BKC;
  const long long h3 = ntn * nch * (2LL * PS_PLANE + 4), x6 = ntn * nch * 3LL * PS_PLANE;
  return h3 > x6 ? h3 : x6;
}

bool pw_presplit_x6_ok(int Cout, int Cin, long long N) {
  return Cout % PX_BM == 0 && Cout % (16 * P122_QA) == 0 && Cin % X6_BKC == 0 && N > 0 && N <= 0x7fffffffLL &&
         (long long)Cin * N * 4 <= 0x7fffffffffffLL;
}

// a: the pointwise conv as conv_launch would run it on cfg 122 in x6 (K = 1, stride 1, one batch item, x [Cin][N],
// y [Cout][N]); w packed for cfg 122 (P = 3).  ws: pw_presplit_bytes(Cin, N) bytes (the three planes).
int pw_presplit_x6_launch(ConvArgs& a, void* ws, hipStream_t st) {
  if (a.K != 1 || a.s != 1 || a.d != 1 || a.pl != 0 || a.ps || !ws) return BC_ERR_ARG;
  if (!pw_presplit_x6_ok(a.Cout, a.Cin, a.Nout) || a.Tin != a.Nout) return BC_ERR_UNSUPPORTED;
  const long long N = a.Nout;
  const int ntn = (int)((N + PS_BN - 1) / PS_BN), nch = a.Cin / X6_BKC;
  unsigned char* planes = reinterpret_cast<unsigned char*>(ws);
  {
    LTScope lt("presplit_b_x6_kernel", 0.0, (4.0 + 6.0) * a.Cin * (double)N, st);  // fp32 in, three bf16 planes out
    hipLaunchKernelGGL(presplit_b_x6_kernel, dim3(ntn), dim3(256), 0, st, a.x, planes, a.Cin, (int)N, nch);
    BC_CHECK_LAUNCH();
  }
  a.vec = conv_epilogue_vec_ok(a);
  a.ntm = a.Cout / PX_BM;
  a.ntn = ntn;
  a.nchunks = nch;
  const long long nwg = (long long)a.ntm * ntn;
  if (nwg > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  a.nwg = (int)nwg;
  a.wsc = nullptr;
  LTScope lt("pw_presplit_x6_kernel", 2.0 * a.Cout * (double)a.Cin * N, (6.0 * a.Cin + 4.0 * a.Cout) * (double)N, st);
  hipLaunchKernelGGL(pw_presplit_x6_kernel, dim3(a.nwg), dim3(1024), PX_LDS, st, a, planes);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

bool pw_presplit_ok(int Cout, int Cin, long long N) {
  return Cout % (16 * PS_MT * PS_WM) == 0 && Cin % X6_BKC == 0 && N > 0 && N <= 0x7fffffffLL &&
         (long long)Cin * N * 4 <= 0x7fffffffffffLL;
}

// a: the pointwise conv as conv_launch would run it on cfg 322 (K = 1, stride 1, one batch item, x [Cin][N],
// y [Cout][N]); w packed for cfg 322.  ws: pw_presplit_bytes(Cin, N) bytes (planes, then the scales).
int pw_presplit_launch(ConvArgs& a, void* ws, hipStream_t st) {
  if (a.K != 1 || a.s != 1 || a.d != 1 || a.pl != 0 || a.ps || !ws) return BC_ERR_ARG;
  if (!pw_presplit_ok(a.Cout, a.Cin, a.Nout) || a.Tin != a.Nout) return BC_ERR_UNSUPPORTED;
  const long long N = a.Nout;
  const int ntn = (int)((N + PS_BN - 1) / PS_BN), nch = a.Cin / X6_BKC;
  unsigned char* planes = reinterpret_cast<unsigned char*>(ws);
  float* scales = reinterpret_cast<float*>(planes + (long long)ntn * nch * 2 * PS_PLANE);
  {
    LTScope lt("presplit_b_kernel", 0.0, (4.0 + 4.0) * a.Cin * (double)N, st);  // fp32 in, two fp16 planes out
    hipLaunchKernelGGL(presplit_b_kernel, dim3(ntn), dim3(256), 0, st, a.x, planes, scales, a.Cin, (int)N, nch);
    BC_CHECK_LAUNCH();
  }
  a.vec = conv_epilogue_vec_ok(a);
  a.ntm = a.Cout / (16 * PS_MT * PS_WM);
  a.ntn = ntn;
  a.nchunks = nch;
  const long long nwg = (long long)a.ntm * ntn;
  if (nwg > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  a.nwg = (int)nwg;
  a.wsc = reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(a.w) +
                                         (long long)a.ntm * nch * PS_APIECES * 1024);  // 1 / row scales after the planes
  LTScope lt("pw_presplit_kernel", 2.0 * a.Cout * (double)a.Cin * N, (4.0 * a.Cin + 4.0 * a.Cout) * (double)N, st);
  hipLaunchKernelGGL(pw_presplit_kernel, dim3(a.nwg), dim3(1024), PS_LDS, st, a, planes, scales);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

}  // namespace bc

BC_DEBUG_EXPORT(pw_presplit)
