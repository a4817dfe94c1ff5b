// Weight-normed Conv1d / ConvTranspose1d as implicit-im2col fp32 MFMA GEMMs for gfx950.
//
// Reference: vq/module.py:11-48 (CausalConv1d), :50-57 (CausalConvTranspose1d), :59-72 (WNConv1d /
// WNConvTranspose1d), used by ResidualUnit (:74-89), EncoderBlock (:91-113), DecoderBlock
// (:115-141), BigCodecEncoder (vq/codec_encoder.py:35-57) and BigCodecDecoder
// (vq/codec_decoder.py:59-81).  The weight-norm fold w = g*v/||v|| happens once on the host.
//
// GEMM view of one conv:  y[b,co,n] = bias[co] + sum_{ci,k} W[co,ci,k] * x[b,ci, n*s + k*d - pl]
//   M = Cout, N = output positions of one clip, K = Cin*taps.
// Epilogue (fused): + bias, + residual (ResidualUnit's `x + block(x)`), then either tanh (decoder
// tail) or the SnakeBeta of the NEXT Activation1d (per output channel) — written alone, or beside
// the raw value when the raw value is still needed as a residual (dual output).  Moving every Snake
// into the producing conv's epilogue computes it exactly once per element and keeps the operand
// staging a pure copy.
//
// Matrix core: v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulate).  One 256-thread
// workgroup computes a BM x BN output tile of one clip: WM x WN waves, each MT x NT 16x16 tiles.
// K is walked in chunks of BKC input channels; inside a chunk k is tap-major (k = tap*BKC + ci) so
// one MFMA k-step (4 values) covers 4 channels of one tap.  Both operand tiles of a chunk are
// copied HBM/L2 -> LDS by LDS-DMA into one of two stages while the other stage feeds the MFMAs
// (one barrier per chunk):
//   A (weights): packed [kstep][wave_m][lane] float4, global_load_lds_dwordx4 (1 KiB pieces)
//   B (input)  : [ci][pitch] rows incl. the stride/dilation halo, buffer_load_dword ... lds with
//                out-of-range lanes redirected past the buffer end so the hardware returns 0
//                (zero padding for free).  pitch is chosen so the two 16-lane row groups of a
//                ds_read_b32 half-wave hit disjoint banks.
// ConvTranspose1d runs as `stride` polyphase convolutions whose outputs are written with output
// stride `s` (bc_convT1d_fwd in abi.hip).
#include <cstdio>

#include "bc_common.h"
#include "bc_internal.h"
#include "conv_epilogue.h"

namespace bc {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ lds_ptr_t to_lds(const float* p) {
  return (lds_ptr_t)(p);
}

template <int MT, int WM, int NT, int WN, int BKC>
__global__ void __launch_bounds__(256) conv1d_mfma_kernel(ConvArgs a) {
  constexpr int BM = 16 * MT * WM;
  constexpr int BN = 16 * NT * WN;
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int nks = BKC * a.K / 4;
  const int stage_floats = a.astage + a.bstage;

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

  // Buffer descriptor of this clip's input; its inputs are made provably wave-uniform
  // (readfirstlane) so hipcc emits plain buffer loads instead of waterfall loops (guide T20).
  const unsigned long long xb_u = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned xb_lo = __builtin_amdgcn_readfirstlane((unsigned)xb_u);
  const unsigned xb_hi = __builtin_amdgcn_readfirstlane((unsigned)(xb_u >> 32));
  const int xbytes = __builtin_amdgcn_readfirstlane(a.Cin * a.Tin * 4);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long long)xb_hi << 32) | xb_lo), 0, xbytes, 0x00020000);
  const int in0 = n0 * a.s - a.pl;
  const long long mg0 = (long long)mt_idx * WM;
  const int a_pieces = nks * WM;                 // 1 KiB each
  const int b_pieces = a.bstage >> 6;            // 64 floats each

  // Issue every LDS-DMA of chunk c into stage st.
  auto issue = [&](int st, int c) {
    float* As = smem + st * stage_floats;
    float* Bs = As + a.astage;
    const floatx4* wsrc = reinterpret_cast<const floatx4*>(a.w) + (mg0 * a.nchunks + c) * (long long)(nks * 64);
    for (int q = wave; q < a_pieces; q += 4) {
      const int ks = q / WM, wm_ = q - ks * WM;
      const floatx4* src = wsrc + (long long)wm_ * a.nchunks * (nks * 64) + ks * 64 + lane;
      __builtin_amdgcn_global_load_lds((const void*)src, to_lds(As + q * 256), 16, 0, 0);
    }
    const int c0 = c * BKC;
    for (int p = wave; p < b_pieces; p += 4) {
      const int f = p * 64 + lane;
      int row = (int)(((float)f + 0.5f) * a.inv_win);
      const int col = f - row * a.win;
      const int ci = c0 + row;
      const int ti = in0 + col;
      const bool ok = row < BKC && ci < a.Cin && ti >= 0 && ti < a.Tin;
      const unsigned voff = ok ? (unsigned)((ci * a.Tin + ti) * 4) : 0xfffffff0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, to_lds(Bs + p * 64), 4, voff, 0, 0, 0);
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int lane_off = ((lane & 15) + wn * NT * 16) * a.s;
  const int krow = lane >> 4;

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int c = 0; c < a.nchunks; ++c) {
    const int st = c & 1;
    if (c + 1 < a.nchunks) issue(st ^ 1, c + 1);
    const floatx4* As = reinterpret_cast<const floatx4*>(smem + st * stage_floats);
    const float* Bs = smem + st * stage_floats + a.astage;
    for (int ks = 0; ks < nks; ++ks) {
      const int kidx = ks * 4;
      const int tap = kidx / BKC;
      const int cb = kidx - tap * BKC;
      const floatx4 av = As[(ks * WM + wm) * 64 + lane];
      const float* xrow = Bs + (cb + krow) * a.win + tap * a.d + lane_off;
      float bv[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[j] = xrow[j * 16 * a.s];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          // operands swapped: the tile comes out transposed (positions x channels), see
          // conv_epilogue.h
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[j], av[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  conv_epilogue<MT, NT>(a, acc, b, m0 + wm * MT * 16, n0 + wn * NT * 16, lane);
}

// ------------------------------------------------------------------------------------------------
// Host side: tile-config table, weight packing, launch.
// cfg id = tile * 4 + bkc_index; tile by Cout, BKC (input channels per K chunk) by shape.
// ------------------------------------------------------------------------------------------------
struct Tile {
  int MT, WM, NT, WN;
};
static const Tile kTiles[] = {
    {4, 2, 4, 2},  // 0: BM=128 BN=128   (Cout >= 128)
    {4, 1, 4, 4},  // 1: BM=64  BN=256
    {3, 1, 4, 4},  // 2: BM=48  BN=256
    {2, 1, 4, 4},  // 3: BM=32  BN=256
    {1, 1, 4, 4},  // 4: BM=16  BN=256
};
static const int kBKC[] = {32, 16, 8, 4};
// Bytes per LDS stage (two stages per workgroup).  BC_STAGE_BUDGET_KB overrides it for tuning
// experiments; weight packing and launch read the same value, so they always agree in-process.
static int stage_budget() {
  static int v = [] {
    const char* e = getenv("BC_STAGE_BUDGET_KB");
    // 32 KB measured best on MI355X (profiles/r01_stage_budget_sweep.txt: 16/24/32/40/56 KB ->
    // 568/562/561/603/698 ms per config-2 step): 2 stages x 32 KB keeps 2 workgroups per CU.
    const int kb = e ? atoi(e) : 32;
    return (kb >= 8 && kb <= 78 ? kb : 32) * 1024;
  }();
  return v;
}

static inline int tile_BM(const Tile& t) { return 16 * t.MT * t.WM; }
static inline int tile_BN(const Tile& t) { return 16 * t.NT * t.WN; }

// Input-tile row pitch: covers (BN-1)*s + (K-1)*d + 1 columns, padded so the two 16-lane row
// groups of a ds_read_b32 half-wave land on disjoint banks (bank = dword index mod 32).
static int choose_pitch(int need, int s) {
  int best = need, best_conf = 1 << 30;
  for (int pad = 0; pad < 32; ++pad) {
    const int w = need + pad;
    int cnt[32] = {0};
    for (int l = 0; l < 32; ++l) cnt[((l >> 4) * w + (l & 15) * s) & 31]++;
    int conf = 0;
    for (int k = 0; k < 32; ++k) conf = conf > cnt[k] ? conf : cnt[k];
    if (conf < best_conf) {
      best_conf = conf;
      best = w;
    }
    if (conf == 1) break;
  }
  return best;
}

static inline int round_up(int v, int m) { return (v + m - 1) / m * m; }

struct Geometry {
  int pitch, bstage, astage, nks;
};
static Geometry geometry(const Tile& t, int bkc, int K, int s, int d) {
  Geometry g;
  g.pitch = choose_pitch((tile_BN(t) - 1) * s + (K - 1) * d + 1, s);
  g.bstage = round_up(bkc * g.pitch, 64);
  g.nks = bkc * K / 4;
  g.astage = g.nks * t.WM * 256;
  return g;
}

int conv_select_cfg(int Cout, int Cin, int K, int stride, int dilation, int mode) {
  if (mode >= 1 && mode <= 3) {
    const int c = x6_select_cfg(Cout, Cin, K, stride, dilation, mode == 1 ? 3 : mode == 2 ? 1 : 2);
    if (c >= 0) return c;
  }
  int tile;
  if (Cout >= 128) tile = 0;
  else if (Cout > 48) tile = 1;
  else if (Cout > 32) tile = 2;
  else if (Cout > 16) tile = 3;
  else tile = 4;
  const Tile& t = kTiles[tile];
  for (int bi = 0; bi < 4; ++bi) {
    const int bkc = kBKC[bi];
    if (bkc > 4 && bkc > round_up(Cin, 4)) continue;  // do not pad the channel chunk past Cin
    const Geometry g = geometry(t, bkc, K, stride, dilation);
    if (g.nks > 40) continue;
    if ((g.astage + g.bstage) * 4 <= stage_budget()) return tile * 4 + bi;
  }
  return tile * 4 + 3;  // BKC = 4 always fits the shapes the codec builds
}

bool conv_cfg_valid(int cfg_id) { return (cfg_id >= 0 && cfg_id < 20) || x6_cfg_valid(cfg_id); }

long long conv_packed_floats(int Cout, int Cin, int K, int cfg_id) {
  if (x6_cfg_valid(cfg_id)) return x6_packed_bytes(Cout, Cin, K, cfg_id) / 4;
  const Tile& t = kTiles[cfg_id / 4];
  const int bkc = kBKC[cfg_id % 4];
  const int ntm = (Cout + tile_BM(t) - 1) / tile_BM(t);
  const int nchunks = (Cin + bkc - 1) / bkc;
  const int nks = bkc * K / 4;
  return (long long)ntm * t.WM * nchunks * nks * 64 * 4;
}

// w: [Cout][Cin][K] row-major fp32 (host).  out: conv_packed_floats() floats (host).
// Layout: [mgroup][chunk][kstep][lane][4]; mgroup = 16*MT output rows; element i of the float4 is
// m-tile i (zero for i >= MT); lane -> (row = lane&15, k = 4*kstep + (lane>>4)), k tap-major.
void conv_pack_weight(const float* w, float* out, int Cout, int Cin, int K, int cfg_id) {
  if (x6_cfg_valid(cfg_id)) {
    x6_pack_weight(w, reinterpret_cast<unsigned short*>(out), Cout, Cin, K, cfg_id);
    return;
  }
  const Tile& t = kTiles[cfg_id / 4];
  const int bkc = kBKC[cfg_id % 4];
  const int ntm = (Cout + tile_BM(t) - 1) / tile_BM(t);
  const int nmg = ntm * t.WM;
  const int nchunks = (Cin + bkc - 1) / bkc;
  const int nks = bkc * K / 4;
  long long o = 0;
  for (int mg = 0; mg < nmg; ++mg)
    for (int c = 0; c < nchunks; ++c)
      for (int ks = 0; ks < nks; ++ks)
        for (int lane = 0; lane < 64; ++lane)
          for (int i = 0; i < 4; ++i, ++o) {
            float v = 0.f;
            if (i < t.MT) {
              const int row = mg * 16 * t.MT + i * 16 + (lane & 15);
              const int kidx = ks * 4 + (lane >> 4);
              const int tap = kidx / bkc;
              const int ci = c * bkc + (kidx % bkc);
              if (row < Cout && ci < Cin) v = w[((long long)row * Cin + ci) * K + tap];
            }
            out[o] = v;
          }
}

template <int MT, int WM, int NT, int WN, int BKC>
static int launch_tile(ConvArgs& a, int B, hipStream_t st) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  const Tile t{MT, WM, NT, WN};
  const Geometry g = geometry(t, BKC, a.K, a.s, a.d);
  a.ntm = (a.Cout + BM - 1) / BM;
  a.ntn = (a.Nout + BN - 1) / BN;
  a.nchunks = (a.Cin + BKC - 1) / BKC;
  a.win = g.pitch;
  a.inv_win = 1.0f / (float)g.pitch;
  a.bstage = g.bstage;
  a.astage = g.astage;
  const long long nwg = (long long)a.ntm * a.ntn * B;
  if (nwg <= 0) return BC_OK;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  if ((long long)a.Cin * a.Tin * 4 > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;  // buffer range
  a.nwg = (int)nwg;
  const size_t lds = (size_t)2 * (g.astage + g.bstage) * 4;
  if (lds > 160 * 1024) return BC_ERR_UNSUPPORTED;
  hipLaunchKernelGGL((conv1d_mfma_kernel<MT, WM, NT, WN, BKC>), dim3(a.nwg), dim3(256), lds, st, a);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

#define BC_TILE_CASES(T, MT, WM, NT, WN)                              \
  case T * 4 + 0: return launch_tile<MT, WM, NT, WN, 32>(a, B, st);   \
  case T * 4 + 1: return launch_tile<MT, WM, NT, WN, 16>(a, B, st);   \
  case T * 4 + 2: return launch_tile<MT, WM, NT, WN, 8>(a, B, st);    \
  case T * 4 + 3: return launch_tile<MT, WM, NT, WN, 4>(a, B, st);

int conv_kernel_name(int cfg_id, int K, int s, int d, char* buf, int n) {
  if (x6_cfg_valid(cfg_id)) return x6_kernel_name(cfg_id, K, s, d, buf, n);
  if (!conv_cfg_valid(cfg_id)) return -1;
  const Tile& t = kTiles[cfg_id / 4];
  return snprintf(buf, n, "conv1d_mfma_kernel<%d, %d, %d, %d, %d>", t.MT, t.WM, t.NT, t.WN, kBKC[cfg_id % 4]);
}

int conv_launch(ConvArgs& a, int B, int cfg_id, hipStream_t st) {
  a.vec = conv_epilogue_vec_ok(a);
  if (x6_cfg_valid(cfg_id)) return x6_launch(a, B, cfg_id, st);
  switch (cfg_id) {
    BC_TILE_CASES(0, 4, 2, 4, 2)
    BC_TILE_CASES(1, 4, 1, 4, 4)
    BC_TILE_CASES(2, 3, 1, 4, 4)
    BC_TILE_CASES(3, 2, 1, 4, 4)
    BC_TILE_CASES(4, 1, 1, 4, 4)
  }
  return BC_ERR_ARG;
}
#undef BC_TILE_CASES

}  // namespace bc

BC_DEBUG_EXPORT(conv1d)
