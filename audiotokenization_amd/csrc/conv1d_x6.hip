// Conv1d with fp32-accurate "3 x bf16" MFMA (x6 mode) for gfx950.
//
// Same GEMM and epilogue as conv1d.hip (reference: vq/module.py:11-72 and its callers), but the
// products run on v_mfma_f32_16x16x32_bf16 (16x the fp32 MFMA rate) with every fp32 operand split
// EXACTLY into three bf16 terms, v = v0 + v1 + v2 (round-to-nearest splits; 8+8+8 significant bits
// hold all 24 of an fp32 mantissa).  a*b is accumulated as the six terms with i+j <= 2:
//   a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0
// Every bf16*bf16 product is exact in fp32 and the MFMA accumulates in fp32; the three dropped terms
// are below 2^-26 |ab|.  The result has fp32-level error (DESIGN.md §4 measures it against fp64
// next to native fp32 accumulation) at 6/16 of the fp32-MFMA cost.
//
// Workgroup: 512 threads = WM x WN waves, each MT x NT 16x16 tiles; BM = 16*MT*WM, BN = 16*NT*WN.
// K is walked per (32-channel chunk, tap) = one K32 step.
//   A (weights): split and packed on the host, [mgroup][chunk][tap][plane][m-tile][lane][8 bf16];
//                one step's block (3 planes x WM*MT KiB) is copied by LDS-DMA, double-buffered.
//   B (input)  : per chunk, rows of the tile (incl. stride/dilation halo) are read from HBM into
//                registers (buffer loads: out-of-range -> 0), split into 3 bf16 planes and written
//                channel-contiguous ([col][32 ch], 80-B pitch: conflict-free b128 reads at stride 1)
//                so one ds_read_b128 gives a lane its 8 k-values.  The next chunk's loads are issued
//                at tap 0 and land while the current chunk's taps compute.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "bc_common.h"
#include "bc_internal.h"
#include "conv_epilogue.h"
#include "x6_common.h"

namespace bc {

// P = operand planes: 3 (x6, fp32-accurate), 2 ("h3": two fp16 planes, three products, fp32-class
// accuracy at half the x6 MFMA count, x6_common.h) or 1 (plain bf16 products: the "bf16" precision
// mode of BASELINE config 5, activations still stored fp32).
// h3 scaling: each staged 32-channel B chunk gets a power-of-two scale from its block maximum (a wave
// reduction + an LDS exchange folded into the barrier in front of the chunk's store); the scale only
// ever decreases within a workgroup, the accumulator is rescaled (exactly) when it does, and the
// epilogue multiplies by 1 / (x scale * per-row weight scale).
// PW: pointwise (K = 1, the input tile is exactly BN columns) with the two-chunk-deep B prefetch.
template <int MT, int NT, int WM, int WN, int P, bool PW>
// NT == 1 tiles fit 128 VGPRs without spills: two 512-thread workgroups per CU where LDS allows, so
// one workgroup's epilogue stores and operand loads overlap the other's MFMAs.
__global__ void __launch_bounds__(512, (NT == 1 ? 4 : 2)) conv1d_x6_kernel(ConvArgs a) {
  constexpr int BM = 16 * MT * WM;
  constexpr int BN = 16 * NT * WN;
  constexpr int QA = WM * MT;  // m-tiles per workgroup (1 KiB per plane each)
  constexpr int CI = PW ? BN / 32 : X6_MAXCOL_ITERS;  // 32-column B passes per chunk
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_x6[];
  __shared__ unsigned smax[2][8];  // P == 2: per-wave maxima of the staged B chunk, by chunk parity
  typedef typename FragType<P>::type frag_t;

  const int ncol = a.win;                // columns of the input tile
  const int bplane = a.bstage;           // bytes per B plane (multiple of 16)
  unsigned char* Bs = smem_x6;                            // [3][ncol][80 B]
  unsigned char* As = smem_x6 + P * bplane;               // [2][P][QA][1 KiB]

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int mt_idx = wg % a.ntm;
  const int rest = wg / a.ntm;
  const int nt_idx = rest % a.ntn;
  const int b = rest / a.ntn;
  const int m0 = mt_idx * BM;
  const int n0 = nt_idx * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM;
  const int wn = wave / WM;

  const unsigned long long xb_u = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned xb_lo = __builtin_amdgcn_readfirstlane((unsigned)xb_u);
  const unsigned xb_hi = __builtin_amdgcn_readfirstlane((unsigned)(xb_u >> 32));
  const int xbytes = __builtin_amdgcn_readfirstlane((a.ps ? a.cin0 : a.Cin) * a.Tin * 4);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long long)xb_hi << 32) | xb_lo), 0, xbytes, 0x00020000);
  const int in0 = n0 * a.s - a.pl;
  const int tstep = a.ps ? a.ps : 1;  // input samples per B-tile column

  const int K = a.K;
  const int nsteps = a.nchunks * K;
  const int a_pieces = P * QA;
  const unsigned char* wblk = reinterpret_cast<const unsigned char*>(a.w) +
                              (long long)mt_idx * a.nchunks * K * (a_pieces * 1024);

  auto issue_a = [&](int step, int buf) {
    const unsigned char* src = wblk + (long long)step * (a_pieces * 1024);
    unsigned char* dst = As + buf * (a_pieces * 1024);
    for (int q = wave; q < a_pieces; q += 8)
      __builtin_amdgcn_global_load_lds((const void*)(src + q * 1024 + lane * 16), (lds_void_t)(dst + q * 1024),
                                       16, 0, 0);
  };

  // B staging: thread -> (channel pair p, column lane cl); columns cl + 32*i, i < CI
  const int bp = tid >> 5;       // 0..15
  const int bcl = tid & 31;
  float bv0[CI], bv1[CI];
  auto load_b = [&](int chunk, float (&v0)[CI], float (&v1)[CI]) {
    const int ci0 = chunk * X6_BKC + 2 * bp;
    // channel (row) -> input channel and the input time of column 0; phase mode: row ci' is phase
    // r = ci' % ps of channel ci' / ps, column m reads sample (n0 + m) * ps + r - pl
    int ch0 = ci0, ch1 = ci0 + 1, tb0 = in0, tb1 = in0;
    if (a.ps) {
      ch0 = ci0 / a.ps;
      ch1 = (ci0 + 1) / a.ps;
      tb0 = n0 * a.ps + (ci0 - ch0 * a.ps) - a.pl;
      tb1 = n0 * a.ps + (ci0 + 1 - ch1 * a.ps) - a.pl;
    }
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcl + 32 * i;
      const int t0 = tb0 + col * tstep, t1 = tb1 + col * tstep;
      const bool cin = col < ncol;
      const unsigned o0 = (cin && ci0 < a.Cin && t0 >= 0 && t0 < a.Tin) ? (unsigned)((ch0 * a.Tin + t0) * 4) : 0xfffffff0u;
      const unsigned o1 =
          (cin && ci0 + 1 < a.Cin && t1 >= 0 && t1 < a.Tin) ? (unsigned)((ch1 * a.Tin + t1) * 4) : 0xfffffff0u;
      v0[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o0, 0, 0));
      v1[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o1, 0, 0));
    }
  };
  // P == 2: publish this wave's block maximum of a chunk's staged values / read the block's scale
  auto bmax_publish = [&](const float (&w0)[CI], const float (&w1)[CI], int par) {
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const unsigned u0 = __float_as_uint(fabsf(w0[i])), u1 = __float_as_uint(fabsf(w1[i]));
      m = m > u0 ? m : u0;
      m = m > u1 ? m : u1;
    }
    m = wave_max_u32(m);
    if (lane == 0) smax[par][wave] = m;
  };
  auto bmax_scale = [&](int par) {
    unsigned m = smax[par][0];
#pragma unroll
    for (int w = 1; w < 8; ++w) m = m > smax[par][w] ? m : smax[par][w];
    return h3_scale_from_bits(__builtin_amdgcn_readfirstlane(m));
  };
  float xs = 1.f;  // P == 2: scale of the staged chunk and of the accumulator
  auto store_b = [&](const float (&w0)[CI], const float (&w1)[CI]) {
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcl + 32 * i;
      if (col < ncol) {
        const float v0 = w0[i], v1 = w1[i];
        if constexpr (P == 2) {
          unsigned h, m;
          split2_h(v0 * xs, v1 * xs, h, m);
          unsigned char* p = Bs + col * X6_PITCH + bp * 4;
          *reinterpret_cast<unsigned*>(p) = h;
          *reinterpret_cast<unsigned*>(p + bplane) = m;
          continue;
        }
        const unsigned h = pk_bf16(v0, v1);
        unsigned char* p = Bs + col * X6_PITCH + bp * 4;
        *reinterpret_cast<unsigned*>(p) = h;
        if (P == 3) {
          const float r0 = v0 - bf_lo(h), r1 = v1 - bf_hi(h);
          const unsigned m = pk_bf16(r0, r1);
          const float s0 = r0 - bf_lo(m), s1 = r1 - bf_hi(m);
          const unsigned l = pk_bf16(s0, s1);
          *reinterpret_cast<unsigned*>(p + bplane) = m;
          *reinterpret_cast<unsigned*>(p + 2 * bplane) = l;
        }
      }
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // P == 2, at a chunk boundary (the previous chunk's B tile is no longer read): the next chunk's
  // scale = min(current, its block scale); the accumulator follows exactly (powers of two)
  auto h3_next_scale = [&](int par) {
    const float sn = bmax_scale(par);
    if (sn < xs) {
      const float r = sn / xs;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] *= r;
      xs = sn;
    }
  };

  const int col_lane = (wn * NT * 16 + (lane & 15)) * a.s;
  const int kgrp16 = (lane >> 4) * 16;

  // one K32 step: this wave's MT x NT tiles += A(step) * B(tap-shifted columns)
  auto compute = [&](int step, int tap) {
      const unsigned char* Ab = As + (step & 1) * (a_pieces * 1024);
      const unsigned char* Bcol = Bs + (col_lane + tap * a.d) * X6_PITCH + kgrp16;
      frag_t bf[NT][P];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int p = 0; p < P; ++p)
          bf[j][p] = *reinterpret_cast<const frag_t*>(Bcol + j * 16 * a.s * X6_PITCH + p * bplane);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const unsigned char* Aq = Ab + (wm * MT + i) * 1024 + lane * 16;
        const frag_t a0 = *reinterpret_cast<const frag_t*>(Aq);
        if constexpr (P == 2) {
          const frag_t a1 = *reinterpret_cast<const frag_t*>(Aq + QA * 1024);
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            floatx4 t = acc[i][j];
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][1], a0, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][0], a1, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][0], a0, t, 0, 0, 0);
            acc[i][j] = t;
          }
          continue;
        } else {
        if (P == 1) {
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a0, acc[i][j], 0, 0, 0);
          continue;
        }
        const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(Aq + QA * 1024);
        const bf16x8_t a2 = *reinterpret_cast<const bf16x8_t*>(Aq + 2 * QA * 1024);
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          // operands swapped (input as A): the tile comes out transposed, see conv_epilogue.h
          floatx4 t = acc[i][j];
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a2, t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a1, t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][P - 1], a0, t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a1, t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a0, t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a0, t, 0, 0, 0);
          acc[i][j] = t;
        }
        }
      }
  };

  // prologue: A(step 0), B(chunk 0)
  issue_a(0, 0);
  load_b(0, bv0, bv1);
  if constexpr (P == 2) {
    bmax_publish(bv0, bv1, 0);
    lds_barrier();
    xs = bmax_scale(0);
  }
  store_b(bv0, bv1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  if constexpr (PW) {
    // Pointwise conv (K = 1): one step per chunk, so the B loads run two chunks ahead in two
    // register sets (chunk c + 2 is issued while chunk c computes and chunk c + 1 is stored).
    float bw0[CI], bw1[CI];
    if (a.nchunks > 1) load_b(1, bw0, bw1);
    auto step1 = [&](int c, const float (&n0v)[CI], const float (&n1v)[CI], float (&p0v)[CI], float (&p1v)[CI]) {
      if (c + 1 < a.nchunks && !(a.dbg & 1)) issue_a(c + 1, (c + 1) & 1);
      if (c + 2 < a.nchunks && !(a.dbg & 2)) load_b(c + 2, p0v, p1v);
      compute(c, 0);
      if (c + 1 < a.nchunks) {
        if constexpr (P == 2) bmax_publish(n0v, n1v, (c + 1) & 1);
        lds_barrier();  // every wave is done reading this chunk's B tile
        if constexpr (P == 2) h3_next_scale((c + 1) & 1);
        if (!(a.dbg & 4)) store_b(n0v, n1v);
      }
      // the A copy of step c + 1 (issued before the 2*CI loads of chunk c + 2) must have landed
      if (c + 2 < a.nchunks)
        wait_vmcnt<2 * CI>();
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
    };
    for (int c = 0; c < a.nchunks; c += 2) {
      step1(c, bw0, bw1, bv0, bv1);
      if (c + 1 < a.nchunks) step1(c + 1, bv0, bv1, bw0, bw1);
    }
  } else {
    for (int c = 0; c < a.nchunks; ++c) {
      for (int tap = 0; tap < K; ++tap) {
        const int step = c * K + tap;
        if (step + 1 < nsteps && !(a.dbg & 1)) issue_a(step + 1, (step + 1) & 1);
        if (tap == 0 && c + 1 < a.nchunks && !(a.dbg & 2)) load_b(c + 1, bv0, bv1);
        compute(step, tap);
        if (tap == K - 1 && c + 1 < a.nchunks) {
          if constexpr (P == 2) bmax_publish(bv0, bv1, (c + 1) & 1);
          lds_barrier();  // every wave is done reading this chunk's B tile
          if constexpr (P == 2) h3_next_scale((c + 1) & 1);
          if (!(a.dbg & 4)) store_b(bv0, bv1);
        }
        // Only the next step's A copy (LDS-DMA, not tracked by the compiler) must have landed.  At
        // tap 0 of a multi-tap chunk the 2*CI B loads of the next chunk were issued after it and
        // may stay in flight (vmcnt retires in issue order); they are consumed at the chunk's last
        // tap, where the compiler waits for their registers itself.
        if (tap == 0 && K > 1 && c + 1 < a.nchunks)
          wait_vmcnt<2 * CI>();
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
      }
    }
  }

  if (!(a.dbg & 8)) {
    if constexpr (P == 2)
      conv_epilogue<MT, NT, true>(a, acc, b, m0 + wm * MT * 16, n0 + wn * NT * 16, lane, 1.f / xs);
    else
      conv_epilogue<MT, NT>(a, acc, b, m0 + wm * MT * 16, n0 + wn * NT * 16, lane);
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
// cfg ids 100..: index into this table
static const X6Tile kX6Tiles[] = {
    {4, 4, 2, 4},  // 100: BM=128 BN=256  (Cout >= 128, stride 1)
    {4, 2, 2, 4},  // 101: BM=128 BN=128  (Cout >= 128, stride 2)
    {4, 2, 4, 2},  // 102: BM=256 BN=64   (Cout >= 256, stride >= 3)
    {2, 2, 4, 2},  // 103: BM=128 BN=64   (Cout >= 128, stride >= 3)
    {6, 2, 1, 8},  // 104: BM=96  BN=256
    {4, 2, 1, 8},  // 105: BM=64  BN=256
    {3, 2, 1, 8},  // 106: BM=48  BN=256
    {2, 2, 1, 8},  // 107: BM=32  BN=256
    {1, 2, 1, 8},  // 108: BM=16  BN=256
    {6, 1, 1, 8},  // 109: BM=96  BN=128
    {4, 1, 1, 8},  // 110: BM=64  BN=128
    {3, 1, 1, 8},  // 111: BM=48  BN=128
    {2, 1, 1, 8},  // 112: BM=32  BN=128
    {1, 1, 1, 8},  // 113: BM=16  BN=128
    {6, 2, 2, 4},  // 114: BM=192 BN=128  (Cout = 192k, stride <= 2)
    {6, 1, 2, 4},  // 115: BM=192 BN=64
    {3, 1, 2, 4},  // 116: BM=96  BN=64   (one-launch ResidualUnit at C = 96, two workgroups per CU)
    {4, 1, 2, 4},  // 117: BM=128 BN=64   (two workgroups per CU)
};
constexpr int X6_NT = sizeof(kX6Tiles) / sizeof(kX6Tiles[0]);

static inline size_t x6_lds(const X6Tile& t, int ncol, int planes) {
  const size_t bplane = (size_t)((ncol * X6_PITCH + 15) / 16 * 16);
  return planes * bplane + 2 * planes * (size_t)t.WM * t.MT * 1024;
}

// cfg ids: 100 + tile (x6, three planes), 200 + tile (bf16, one plane), 300 + tile (h3, two fp16
// planes); + 1000 * s for a stride-s
// conv run by phase decomposition (ConvArgs::ps): the stride-1 conv with ceil(K/s) taps over s * Cin
// phase channels ci' = ci * s + r, weights W'[co][ci'][q] = W[co][ci][q * s + r] (0 past K).  Its
// input tile needs BN + ceil(K/s) - 1 columns instead of (BN - 1) * s + K, so the wide 128 x 256
// tile fits the stride-4/5 convs.
static inline int cfg_base(int cfg) { return cfg % 1000; }
static inline int cfg_phase(int cfg) { return cfg / 1000; }
bool x6_cfg_valid(int cfg) {
  const int b = cfg_base(cfg), s = cfg_phase(cfg);
  return ((b >= 100 && b < 100 + X6_NT) || (b >= 200 && b < 200 + X6_NT) || (b >= 300 && b < 300 + X6_NT)) &&
         (s == 0 || (s >= 2 && s <= 16));
}
// 100..: x6 (3 bf16 planes), 200..: bf16 (1 plane), 300..: h3 (2 fp16 planes + per-row scales)
static inline int cfg_planes(int cfg) {
  const int b = cfg_base(cfg);
  return b >= 300 ? 2 : b >= 200 ? 1 : 3;
}
static inline int planes_base(int planes) { return planes == 1 ? 200 : planes == 2 ? 300 : 100; }
static inline const X6Tile& cfg_tile(int cfg) { return kX6Tiles[cfg_base(cfg) % 100]; }
const X6Tile& x6_tile(int cfg) { return cfg_tile(cfg); }

// Returns a x6 (planes = 3) / bf16 (planes = 1) cfg id, or -1 when the shape should stay on the
// fp32 kernel.
// Two-workgroup-per-CU preference: NT == 1 tiles whose LDS fits twice in a CU let one workgroup's
// operand loads and epilogue stores overlap the other's MFMAs.  Measured on MI355X (profiles/
// r01_occ_sweep.txt): a win for the short-K / small-M convs (Cout <= 384 with Cin*K <= 1536: the
// C = 192 k7 and k1 convs, the C = 384 k1 conv, the stride-2 convs), a loss for the long-K ones.
// BC_X6_OCC (tuning experiments): 4 = always try them first, 2 = never, unset = that rule.
static int x6_occ_pref() {
  static int v = [] {
    const char* e = getenv("BC_X6_OCC");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static int x6_select_tile(int Cout, int Cin, int K, int s, int d, int planes);

// Stride >= 3 convs with dilation 1 (the encoder's k=2s downsampling) run phase-decomposed
// (BC_X6_PHASE=0 disables it for A/B timing).
static bool x6_phase_ok(int s, int d) {
  static int v = [] {
    const char* e = getenv("BC_X6_PHASE");
    return e ? atoi(e) : 1;
  }();
  return v && s >= 3 && s <= 16 && d == 1;
}

// Measured tile preferences of the x6 (three-plane) kernel, from a sweep of every tile over the
// BigCodec encoder's conv shapes (tools/conv_bench.py --cfg all, profiles/r01_tile_sweep.txt):
//   pointwise, Cout % 128 == 0     -> 101 (128 x 128, two-chunk B prefetch): C = 384 / 768 and the
//                                     LSTM input projection 1536 -> 6144, 12-24 % under the others
//   pointwise, Cout % 96 == 0      -> 116 (96 x 64, two workgroups per CU): C = 192
//   stride 1, K > 1, Cout % 96 == 0 and <= 384 -> 109 (96 x 128, all 8 waves on one 96-row block,
//                                     two workgroups per CU): k7 C = 192 -17 %, C = 384 -2 %
//   stride 2, Cout % 96 == 0 and <= 192 -> phase-decomposed 109: the k4 downsampling at C = 48 / 96
//                                     -33 % / -7 %
// Returns the cfg or -1 (then the general rules below decide).
static int x6_preferred_cfg(int Cout, int Cin, int K, int s, int d) {
  auto fits2 = [](int tile, int K_, int s_, int d_) {  // two workgroups per CU: LDS <= 80 KiB
    const X6Tile& t = kX6Tiles[tile];
    const int ncol = x6_ncol(t, K_, s_, d_);
    return ncol <= 32 * X6_MAXCOL_ITERS && x6_lds(t, ncol, 3) <= 80 * 1024;
  };
  if (s == 1 && K == 1) {
    if (Cout % 128 == 0) return 101;
    if (Cout % 96 == 0) return 116;
    return -1;
  }
  if (s == 1 && Cout % 96 == 0 && Cout <= 384 && fits2(9, K, 1, d)) return 109;
  if (s == 2 && d == 1 && Cout % 96 == 0 && Cout <= 192 && Cin * 2 >= 32 && fits2(9, (K + 1) / 2, 1, 1))
    return 2000 + 109;
  return -1;
}

int x6_select_cfg(int Cout, int Cin, int K, int s, int d, int planes) {
  if (Cin < 16) return -1;  // e.g. the first conv (Cin = 1): no K to amortise the split over
  if (planes >= 2 && x6_occ_pref() == 0) {
    const int c = x6_preferred_cfg(Cout, Cin, K, s, d);
    if (c >= 0) return c + (planes == 2 ? 200 : 0);
  }
  if (x6_phase_ok(s, d)) {
    const int c = x6_select_tile(Cout, Cin * s, (K + s - 1) / s, 1, 1, planes);
    if (c >= 0) return 1000 * s + c;
  }
  return x6_select_tile(Cout, Cin, K, s, d, planes);
}

static int x6_select_tile(int Cout, int Cin, int K, int s, int d, int planes) {
  int order[8];
  bool occ4[8] = {false};
  int n = 0;
  const int pref = x6_occ_pref();
  if (pref == 4 || (pref == 0 && Cout <= 384 && Cin * K <= 1536)) {
    int c = -1;
    if (Cout >= 128) c = Cout % 128 == 0 ? 17 : Cout % 96 == 0 ? 16 : -1;
    else {
      const int mt = (Cout + 15) / 16;
      c = mt >= 5 ? 9 : mt == 4 ? 10 : mt == 3 ? 11 : mt == 2 ? 12 : 13;
    }
    if (c >= 0) {
      occ4[n] = true;
      order[n++] = c;
    }
  }
  if (Cout >= 128 && Cout % 128 != 0 && Cout % 192 == 0) {
    // 192-row tiles: no half-empty m-tile at C = 192 / 576
    if (s <= 2) order[n++] = 14;
    order[n++] = 15;
  }
  if (Cout >= 128) {
    if (s == 1) order[n++] = 0;
    if (s <= 2) order[n++] = 1;
    if (Cout >= 256) order[n++] = 2;
    order[n++] = 3;
  } else {
    const int mt = (Cout + 15) / 16;
    const int base = mt == 6 || mt == 5 ? 0 : mt == 4 ? 1 : mt == 3 ? 2 : mt == 2 ? 3 : 4;
    if (mt > 6) return -1;
    order[n++] = 4 + base;
    order[n++] = 9 + base;
  }
  for (int i = 0; i < n; ++i) {
    const X6Tile& t = kX6Tiles[order[i]];
    const int ncol = x6_ncol(t, K, s, d);
    if (ncol > 32 * X6_MAXCOL_ITERS) continue;
    if (x6_lds(t, ncol, planes) > (occ4[i] ? 80 : 160) * 1024) continue;
    return planes_base(planes) + order[i];
  }
  return -1;
}

long long x6_packed_bytes(int Cout, int Cin, int K, int cfg) {
  const X6Tile& t = cfg_tile(cfg);
  if (const int s = cfg_phase(cfg)) {
    Cin *= s;
    K = (K + s - 1) / s;
  }
  const int ntm = (Cout + x6_BM(t) - 1) / x6_BM(t);
  const int nchunks = (Cin + X6_BKC - 1) / X6_BKC;
  const long long planes = (long long)ntm * nchunks * K * cfg_planes(cfg) * t.WM * t.MT * 1024;
  return planes + (cfg_planes(cfg) == 2 ? (long long)ntm * x6_BM(t) * 4 : 0);  // h3: + 1 / row scale
}

static inline unsigned short f2bf_rn(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);  // NaN
  const unsigned r = u + 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(r >> 16);
}
static inline unsigned short f2h_rn(float f) {
  const _Float16 h = (_Float16)f;  // IEEE round-to-nearest-even
  unsigned short u;
  memcpy(&u, &h, 2);
  return u;
}
static inline float h2f(unsigned short u) {
  _Float16 h;
  memcpy(&h, &u, 2);
  return (float)h;
}
static inline float bf2f(unsigned short h) {
  const unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// w: [Cout][Cin][K] fp32 host -> packed bf16 planes (host), layout documented at the top.
void x6_pack_weight(const float* w, unsigned short* out, int Cout, int Cin, int K, int cfg) {
  if (const int s = cfg_phase(cfg)) {  // phase-decomposed weights W'[co][ci * s + r][q]
    const int Kp = (K + s - 1) / s, Cp = Cin * s;
    std::vector<float> wp((size_t)Cout * Cp * Kp, 0.f);
    for (int co = 0; co < Cout; ++co)
      for (int ci = 0; ci < Cin; ++ci)
        for (int k = 0; k < K; ++k)
          wp[((size_t)co * Cp + ci * s + k % s) * Kp + k / s] = w[((size_t)co * Cin + ci) * K + k];
    x6_pack_weight(wp.data(), out, Cout, Cp, Kp, cfg_base(cfg));
    return;
  }
  const X6Tile& t = cfg_tile(cfg);
  const int P = cfg_planes(cfg);
  const int BM = x6_BM(t), QA = t.WM * t.MT;
  const int ntm = (Cout + BM - 1) / BM;
  const int nchunks = (Cin + X6_BKC - 1) / X6_BKC;
  // h3: per-row power-of-two scale 2^(14 - e), 2^e <= max |w[row]| < 2^(e+1) (see x6_common.h)
  std::vector<float> rsc(P == 2 ? (size_t)ntm * BM : 0, 1.f);
  for (size_t row = 0; row < rsc.size() && (int)row < Cout; ++row) {
    float m = 0.f;
    for (long long k = 0; k < (long long)Cin * K; ++k) m = std::max(m, std::fabs(w[(long long)row * Cin * K + k]));
    if (m > 0.f && std::isfinite(m)) {
      const int e = std::max(-112, std::min(140, std::ilogb(m)));
      rsc[row] = std::ldexp(1.f, 14 - e);
    }
  }
  long long o = 0;
  for (int mg = 0; mg < ntm; ++mg)
    for (int c = 0; c < nchunks; ++c)
      for (int tap = 0; tap < K; ++tap)
        for (int p = 0; p < P; ++p)
          for (int q = 0; q < QA; ++q)
            for (int lane = 0; lane < 64; ++lane)
              for (int j = 0; j < 8; ++j, ++o) {
                const int row = mg * BM + q * 16 + (lane & 15);
                const int ci = c * X6_BKC + 8 * (lane >> 4) + j;
                float v = 0.f;
                if (row < Cout && ci < Cin) v = w[((long long)row * Cin + ci) * K + tap];
                if (P == 2) {
                  const float vs = v * rsc[row];
                  const unsigned short g0 = f2h_rn(vs);
                  out[o] = p == 0 ? g0 : f2h_rn(vs - h2f(g0));
                  continue;
                }
                const unsigned short h0 = f2bf_rn(v);
                const float r1 = v - bf2f(h0);
                const unsigned short h1 = f2bf_rn(r1);
                const float r2 = r1 - bf2f(h1);
                const unsigned short h2 = f2bf_rn(r2);
                out[o] = p == 0 ? h0 : p == 1 ? h1 : h2;
              }
  if (P == 2) {  // 1 / row scale after the planes (ConvArgs::wsc)
    float* inv = reinterpret_cast<float*>(out + o);
    for (size_t row = 0; row < rsc.size(); ++row) inv[row] = 1.f / rsc[row];
  }
}

// BC_X6_PW=0 runs pointwise convs on the general kernel (A/B timing).
static bool x6_pw_on() {
  static const bool v = [] {
    const char* e = getenv("BC_X6_PW");
    return !e || atoi(e) != 0;
  }();
  return v;
}

template <int MT, int NT, int WM, int WN, int P>
static int launch_x6(ConvArgs& a, int B, hipStream_t st) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const X6Tile t{MT, NT, WM, WN};
  const int ncol = x6_ncol(t, a.K, a.s, a.d);
  if (ncol > 32 * X6_MAXCOL_ITERS) return BC_ERR_UNSUPPORTED;
  a.ntm = (a.Cout + BM - 1) / BM;
  a.ntn = (a.Nout + BN - 1) / BN;
  a.nchunks = (a.Cin + X6_BKC - 1) / X6_BKC;
  a.win = ncol;
  a.bstage = (ncol * X6_PITCH + 15) / 16 * 16;
  const long long nwg = (long long)a.ntm * a.ntn * B;
  if (nwg <= 0) return BC_OK;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  if ((long long)(a.ps ? a.cin0 : a.Cin) * a.Tin * 4 > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  a.nwg = (int)nwg;
  a.wsc = P == 2 ? reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(a.w) +
                                                  (long long)a.ntm * a.nchunks * a.K * P * t.WM * t.MT * 1024)
                 : nullptr;
  const size_t lds = x6_lds(t, ncol, P);
  if (lds > 160 * 1024) return BC_ERR_UNSUPPORTED;
  if (a.K == 1 && ncol == BN && x6_pw_on())
    hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, true>), dim3(a.nwg), dim3(512), lds, st, a);
  else
    hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, false>), dim3(a.nwg), dim3(512), lds, st, a);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int x6_launch(ConvArgs& a, int B, int cfg, hipStream_t st) {
  static const int dbg = [] {
    const char* e = getenv("BC_X6_DEBUG");
    return e ? atoi(e) : 0;
  }();
  a.dbg = dbg;
  a.ps = 0;
  if (const int s = cfg_phase(cfg)) {  // run as the stride-1 conv over the s phases
    if (a.s != s || a.d != 1 || a.ostride != 1) return BC_ERR_ARG;
    a.ps = s;
    a.cin0 = a.Cin;
    a.Cin *= s;
    a.K = (a.K + s - 1) / s;
    a.s = 1;
    cfg = cfg_base(cfg);
  }
#define BC_X6_CASES(ID, MT, NT, WM, WN)                                \
  case 100 + ID: return launch_x6<MT, NT, WM, WN, 3>(a, B, st);        \
  case 200 + ID: return launch_x6<MT, NT, WM, WN, 1>(a, B, st);        \
  case 300 + ID: return launch_x6<MT, NT, WM, WN, 2>(a, B, st);
  switch (cfg) {
    BC_X6_CASES(0, 4, 4, 2, 4)
    BC_X6_CASES(1, 4, 2, 2, 4)
    BC_X6_CASES(2, 4, 2, 4, 2)
    BC_X6_CASES(3, 2, 2, 4, 2)
    BC_X6_CASES(4, 6, 2, 1, 8)
    BC_X6_CASES(5, 4, 2, 1, 8)
    BC_X6_CASES(6, 3, 2, 1, 8)
    BC_X6_CASES(7, 2, 2, 1, 8)
    BC_X6_CASES(8, 1, 2, 1, 8)
    BC_X6_CASES(9, 6, 1, 1, 8)
    BC_X6_CASES(10, 4, 1, 1, 8)
    BC_X6_CASES(11, 3, 1, 1, 8)
    BC_X6_CASES(12, 2, 1, 1, 8)
    BC_X6_CASES(13, 1, 1, 1, 8)
    BC_X6_CASES(14, 6, 2, 2, 4)
    BC_X6_CASES(15, 6, 1, 2, 4)
    BC_X6_CASES(16, 3, 1, 2, 4)
    BC_X6_CASES(17, 4, 1, 2, 4)
  }
#undef BC_X6_CASES
  return BC_ERR_ARG;
}

}  // namespace bc
