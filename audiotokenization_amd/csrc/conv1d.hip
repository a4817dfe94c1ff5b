// Weight-normed Conv1d / ConvTranspose1d as implicit-im2col fp32 MFMA GEMMs for gfx950.
//
// Reference: vq/module.py:11-48 (CausalConv1d), :50-57 (CausalConvTranspose1d), :59-72 (WNConv1d /
// WNConvTranspose1d), used by ResidualUnit (:74-89), EncoderBlock (:91-113), DecoderBlock
// (:115-141), BigCodecEncoder (vq/codec_encoder.py:35-57) and BigCodecDecoder
// (vq/codec_decoder.py:59-81).  The weight-norm fold w = g*v/||v|| happens once on the host.
//
// GEMM view of one conv:  y[b,co,n] = bias[co] + sum_{ci,k} W[co,ci,k] * act(x[b,ci, n*s + k*d - pl])
//   M = Cout, N = output positions of one clip, K = Cin*taps.
// act() is the optional fused SnakeBeta prologue (the Activation1d that precedes every conv in the
// reference), applied while the input tile is staged into LDS.  Epilogue: + bias, optional residual
// add (ResidualUnit's `x + block(x)`), optional tanh (decoder tail, codec_decoder.py:78-80).
//
// Matrix core: v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulate).  One 256-thread
// workgroup computes a BM x BN output tile of one clip: WM x WN waves, each MT x NT 16x16 tiles.
// K is walked in chunks of BKC input channels; inside a chunk the k index is tap-major
// (k = tap*BKC + ci_local) so one MFMA k-step (4 values) covers 4 channels of one tap.
//   LDS A tile : packed weights, [kstep][wave_m][lane] float4 (one ds_read_b128 per lane per k-step)
//   LDS B tile : snake(x) rows, [ci_local][win] with the stride/dilation halo
// ConvTranspose1d is run as `stride` polyphase 2-tap convolutions whose outputs are written with
// output stride `s` (see bc_convT1d_fwd in abi.cpp).
#include "bc_common.h"
#include "bc_internal.h"

namespace bc {



template <int MT, int WM, int NT, int WN, int BKC, bool SNAKE>
__global__ void __launch_bounds__(256) conv1d_mfma_kernel(ConvArgs a) {
  constexpr int BM = 16 * MT * WM;
  constexpr int BN = 16 * NT * WN;
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int nks = BKC * a.K / 4;
  floatx4* As = reinterpret_cast<floatx4*>(smem);           // [nks][WM][64]
  float* xs = smem + nks * WM * 64 * 4;                      // [BKC][win]

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int mt_idx = wg % a.ntm;
  const int rest = wg / a.ntm;
  const int nt_idx = rest % a.ntn;
  const int b = rest / a.ntn;
  const int m0 = mt_idx * BM;
  const int n0 = nt_idx * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const float* xb = a.x + (long long)b * a.xbs;
  const int in0 = n0 * a.s - a.pl;
  const int xs_elems = BKC * a.win;
  const int a_vecs = nks * WM * 64;
  const long long mg0 = (long long)mt_idx * WM;
  const int lane_off = ((lane & 15) + wn * NT * 16) * a.s;
  const int krow = lane >> 4;

  for (int c = 0; c < a.nchunks; ++c) {
    const int c0 = c * BKC;
    // ---- stage B: snake(x) rows with halo -------------------------------------------------
    for (int e = tid; e < xs_elems; e += 256) {
      const int row = e / a.win;
      const int col = e - row * a.win;
      const int ci = c0 + row;
      const int ti = in0 + col;
      float v = 0.f;
      if (ci < a.Cin && ti >= 0 && ti < a.Tin) {
        v = xb[(long long)ci * a.Tin + ti];
        if constexpr (SNAKE) v = snake(v, a.sa[ci], a.sb[ci]);
      }
      xs[e] = v;
    }
    // ---- stage A: packed weights for this chunk -------------------------------------------
    for (int e = tid; e < a_vecs; e += 256) {
      const int wm_ = e / (nks * 64);
      const int r = e - wm_ * nks * 64;  // ks*64 + lane
      const floatx4* src = reinterpret_cast<const floatx4*>(a.w) +
                           ((mg0 + wm_) * a.nchunks + c) * (long long)(nks * 64) + r;
      const int ks = r >> 6;
      As[(ks * WM + wm_) * 64 + (r & 63)] = *src;
    }
    __syncthreads();
    // ---- MFMA over the chunk --------------------------------------------------------------
    for (int ks = 0; ks < nks; ++ks) {
      const int kidx = ks * 4;
      const int tap = kidx / BKC;
      const int cb = kidx - tap * BKC;
      const floatx4 av = As[(ks * WM + wm) * 64 + lane];
      const float* xr = xs + (cb + krow) * a.win + tap * a.d + lane_off;
      float bv[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) bv[j] = xr[j * 16 * a.s];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // ---- epilogue: C/D map of 16x16x4: col = lane&15 (n), row = (lane>>4)*4 + r (m) ----------
  float* yb = a.y + (long long)b * a.ybs;
  const float* rb = a.res ? a.res + (long long)b * a.rbs : nullptr;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = m0 + wm * MT * 16 + i * 16 + (lane >> 4) * 4 + r;
      if (co >= a.Cout) continue;
      const float bias = a.bias ? a.bias[co] : 0.f;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = n0 + wn * NT * 16 + j * 16 + (lane & 15);
        if (n >= a.Nout) continue;
        const long long yi = (long long)co * a.yT + (long long)n * a.ostride + a.ooff;
        float v = acc[i][j][r] + bias;
        if (rb) v = rb[yi] + v;
        if (a.epi == 1) v = tanhf(v);
        yb[yi] = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Host side: tile-config table, weight packing, launch.
// ------------------------------------------------------------------------------------------------
struct TileCfg {
  int MT, WM, NT, WN, BKC;
};
static const TileCfg kCfgs[] = {
    {4, 2, 4, 2, 8},  // 0: BM=128 BN=128
    {4, 1, 4, 4, 8},  // 1: BM=64  BN=256
    {3, 1, 4, 4, 8},  // 2: BM=48  BN=256
    {2, 1, 4, 4, 8},  // 3: BM=32  BN=256
    {1, 1, 4, 4, 8},  // 4: BM=16  BN=256
    {4, 2, 4, 2, 4},  // 5..9: same tiles, BKC=4 (Cin < 8, e.g. the first conv Cin=1)
    {4, 1, 4, 4, 4},
    {3, 1, 4, 4, 4},
    {2, 1, 4, 4, 4},
    {1, 1, 4, 4, 4},
};

int conv_select_cfg(int Cout, int Cin) {
  int base;
  if (Cout >= 128) base = 0;
  else if (Cout > 48) base = 1;
  else if (Cout > 32) base = 2;
  else if (Cout > 16) base = 3;
  else base = 4;
  return Cin < 8 ? base + 5 : base;
}

static inline int cfg_BM(const TileCfg& t) { return 16 * t.MT * t.WM; }
static inline int cfg_BN(const TileCfg& t) { return 16 * t.NT * t.WN; }

long long conv_packed_floats(int Cout, int Cin, int K, int cfg_id) {
  const TileCfg& t = kCfgs[cfg_id];
  const int ntm = (Cout + cfg_BM(t) - 1) / cfg_BM(t);
  const int nchunks = (Cin + t.BKC - 1) / t.BKC;
  const int nks = t.BKC * K / 4;
  return (long long)ntm * t.WM * nchunks * nks * 64 * 4;
}

// w: [Cout][Cin][K] row-major fp32 (host).  out: conv_packed_floats() floats (host).
// Layout: [mgroup][chunk][kstep][lane][4]; mgroup = 16*MT output rows; element i of the float4 is
// m-tile i (zero for i >= MT); lane -> (row = lane&15, k = 4*kstep + (lane>>4)), k tap-major.
void conv_pack_weight(const float* w, float* out, int Cout, int Cin, int K, int cfg_id) {
  const TileCfg& t = kCfgs[cfg_id];
  const int ntm = (Cout + cfg_BM(t) - 1) / cfg_BM(t);
  const int nmg = ntm * t.WM;
  const int nchunks = (Cin + t.BKC - 1) / t.BKC;
  const int nks = t.BKC * K / 4;
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
              const int tap = kidx / t.BKC;
              const int ci = c * t.BKC + (kidx % t.BKC);
              if (row < Cout && ci < Cin) v = w[((long long)row * Cin + ci) * K + tap];
            }
            out[o] = v;
          }
}

// Input-tile row length: covers (BN-1)*s + (K-1)*d + 1 columns, padded so the two 16-lane row
// groups of a ds_read_b32 half-wave land on disjoint banks (bank = dword index mod 32).
static int choose_win(int need, int s) {
  int best = need, best_conf = 1 << 30;
  for (int pad = 0; pad < 32; ++pad) {
    const int w = need + pad;
    int cnt[32] = {0};
    for (int l = 0; l < 32; ++l) {
      const int addr = (l >> 4) * w + (l & 15) * s;
      cnt[addr & 31]++;
    }
    int conf = 0;
    for (int k = 0; k < 32; ++k) conf = conf > cnt[k] ? conf : cnt[k];
    if (conf < best_conf) { best_conf = conf; best = w; }
    if (conf == 1) break;
  }
  return best;
}

template <int MT, int WM, int NT, int WN, int BKC>
static int launch_cfg(ConvArgs& a, int B, hipStream_t st) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN;
  a.ntm = (a.Cout + BM - 1) / BM;
  a.ntn = (a.Nout + BN - 1) / BN;
  a.nchunks = (a.Cin + BKC - 1) / BKC;
  a.win = choose_win((BN - 1) * a.s + (a.K - 1) * a.d + 1, a.s);
  const long long nwg = (long long)a.ntm * a.ntn * B;
  if (nwg <= 0) return BC_OK;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  a.nwg = (int)nwg;
  const int nks = BKC * a.K / 4;
  const size_t lds = (size_t)nks * WM * 64 * 16 + (size_t)BKC * a.win * 4;
  if (lds > 160 * 1024) return BC_ERR_UNSUPPORTED;
  if (a.sa)
    hipLaunchKernelGGL((conv1d_mfma_kernel<MT, WM, NT, WN, BKC, true>), dim3(a.nwg), dim3(256), lds, st, a);
  else
    hipLaunchKernelGGL((conv1d_mfma_kernel<MT, WM, NT, WN, BKC, false>), dim3(a.nwg), dim3(256), lds, st, a);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int conv_launch(ConvArgs& a, int B, int cfg_id, hipStream_t st) {
  if (a.K * 8 % 4 != 0) return BC_ERR_ARG;
  switch (cfg_id) {
    case 0: return launch_cfg<4, 2, 4, 2, 8>(a, B, st);
    case 1: return launch_cfg<4, 1, 4, 4, 8>(a, B, st);
    case 2: return launch_cfg<3, 1, 4, 4, 8>(a, B, st);
    case 3: return launch_cfg<2, 1, 4, 4, 8>(a, B, st);
    case 4: return launch_cfg<1, 1, 4, 4, 8>(a, B, st);
    case 5: return launch_cfg<4, 2, 4, 2, 4>(a, B, st);
    case 6: return launch_cfg<4, 1, 4, 4, 4>(a, B, st);
    case 7: return launch_cfg<3, 1, 4, 4, 4>(a, B, st);
    case 8: return launch_cfg<2, 1, 4, 4, 4>(a, B, st);
    case 9: return launch_cfg<1, 1, 4, 4, 4>(a, B, st);
  }
  return BC_ERR_ARG;
}

}  // namespace bc
