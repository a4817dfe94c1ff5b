// HBM-bound elementwise / resampling kernels.
//
//  snake_kernel     : SnakeBeta alone (vq/activations.py:107-118) for a standalone Activation1d /
//                     SnakeBeta module call.  Inside the encoder/decoder stacks the Snake is fused
//                     into the following conv's input staging instead (conv1d.hip).
//  aa_snake_kernel  : Activation1d with antialias=True (vq/alias_free_torch/act.py:25-32):
//                     UpSample1d (resample.py:25-33: replicate pad 5, depthwise 12-tap transposed
//                     conv stride 2, x2 gain, crop [15:-15]) -> SnakeBeta -> DownSample1d
//                     (filter.py:86-95: replicate pad (5,6), depthwise 12-tap conv stride 2), fused so
//                     the 2T intermediate never leaves LDS.
//  transpose kernels: [B][C][T] <-> [C][T][B] layouts around the ResLSTM (vq/module.py:160-166).
//  synth_clips      : counter-hash white noise generated in HBM.
//  stream_window    : a causal stream's [carried context | chunk] window (+ Snake) and its next context.
#include <algorithm>
#include "bc_common.h"
#include "bc_internal.h"

namespace bc {

__global__ void snake_kernel(const float* __restrict__ x, const float* __restrict__ sa,
                             const float* __restrict__ sb, float* __restrict__ y, int C, long long T,
                             long long total) {
  // element pairs through the packed Snake (the one every conv epilogue runs); an odd tail alone
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = 2 * ((long long)blockIdx.x * blockDim.x + threadIdx.x); i < total; i += 2 * stride) {
    const int c0 = (int)((i / T) % C);
    if (i + 1 < total) {
      const int c1 = (int)(((i + 1) / T) % C);
      const f32x2 v = snake_pk((f32x2){x[i], x[i + 1]}, (f32x2){sa[c0], sa[c1]}, (f32x2){sb[c0], sb[c1]});
      y[i] = v.x;
      y[i + 1] = v.y;
    } else {
      y[i] = snake(x[i], sa[c0], sb[c0]);
    }
  }
}

// One workgroup = one (b, c) row segment of AA_TILE outputs.
constexpr int AA_TILE = 256;
constexpr int AA_TAPS = 12;

__global__ void __launch_bounds__(256) aa_snake_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ sa,
                                                       const float* __restrict__ sb,
                                                       const float* __restrict__ fup,
                                                       const float* __restrict__ fdown,
                                                       float* __restrict__ y, int C, int T,
                                                       int ntiles) {
  __shared__ float xl[AA_TILE / 2 + AA_TILE + 32];
  __shared__ float sl[2 * AA_TILE + 16];
  __shared__ float fu[AA_TAPS], fd[AA_TAPS];
  const int tile = blockIdx.x % ntiles;
  const long long row = blockIdx.x / ntiles;  // b*C + c
  const int c = (int)(row % C);
  const float* xr = x + row * T;
  float* yr = y + row * T;
  const int t0 = tile * AA_TILE;
  if (threadIdx.x < AA_TAPS) {
    fu[threadIdx.x] = fup[threadIdx.x];
    fd[threadIdx.x] = fdown[threadIdx.x];
  }
  // Down stage needs snake values at up-sample index v in [2*t0-5, 2*t0+2*AA_TILE+5].
  // Up-sample index v (after the [15:-15] crop) = u - 15 where u indexes the transposed-conv
  // output; u = 2*i + k with i indexing the replicate-padded input x_p[i] = x[clamp(i-5)].
  const int vbase = 2 * t0 - 5;
  const int nv = 2 * AA_TILE + 11;
  // input indices needed: i = (v + 15 - k)/2 for k in [0,12): i in [(vbase+4)/2, (vmax+15)/2]
  const int ibase = (vbase + 15 - 11) >> 1;  // floor, vbase+4 may be negative -> arithmetic shift
  const int ni = (nv + 12) / 2 + 2;
  for (int e = threadIdx.x; e < ni; e += 256) {
    int xi = ibase + e - 5;
    xi = xi < 0 ? 0 : (xi >= T ? T - 1 : xi);
    xl[e] = xr[xi];
  }
  __syncthreads();
  const float a = sa[c], ib = sb[c];
  for (int e = threadIdx.x; e < nv; e += 256) {
    int v = vbase + e;
    v = v < 0 ? 0 : (v >= 2 * T ? 2 * T - 1 : v);  // replicate pad of the snake output (down stage)
    const int u = v + 15;
    float acc = 0.f;
    // conv_transpose1d: out[u] = sum_{k: (u-k) even} x_p[(u-k)/2] * f[k]
#pragma unroll
    for (int k = (u & 1); k < AA_TAPS; k += 2) {
      const int i = (u - k) >> 1;
      acc = acc + xl[i - ibase] * fu[k];
    }
    const float up = 2.0f * acc;
    sl[e] = snake(up, a, ib);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < AA_TILE; e += 256) {
    const int t = t0 + e;
    if (t >= T) break;
    // out[t] = sum_k z_p[2t+k] f[k], z_p[j] = s[clamp(j-5)]  -> s index v = 2t+k-5
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < AA_TAPS; ++k) acc = acc + sl[2 * e + k] * fd[k];
    yr[t] = acc;
  }
}

// x[B][C][T] -> y[C][T][B]   (tiles of 32 t x B<=64 per channel)
__global__ void __launch_bounds__(256) btc_to_ctb_kernel(const float* __restrict__ x,
                                                         float* __restrict__ y, int B, int C,
                                                         int T) {
  __shared__ float tl[64][33];
  const int tt = blockIdx.x;  // t-tile of 32
  const int c = blockIdx.y;
  const int bt = blockIdx.z;  // b-tile of 64
  const int t0 = tt * 32, b0 = bt * 64;
  for (int e = threadIdx.x; e < 64 * 32; e += 256) {
    const int bl = e / 32, tl_ = e % 32;
    const int b = b0 + bl, t = t0 + tl_;
    tl[bl][tl_] = (b < B && t < T) ? x[((long long)b * C + c) * T + t] : 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 32; e += 256) {
    const int tl_ = e / 64, bl = e % 64;
    const int b = b0 + bl, t = t0 + tl_;
    if (b < B && t < T) y[((long long)c * T + t) * B + b] = tl[bl][tl_];
  }
}

// out[B][C][T] = act(y[C][T][B] + skip[B][C][T])   (ResLSTM skip, vq/module.py:163-166; act = the
// following Activation1d's Snake when sa != nullptr, fused so the LSTM output is written once)
__global__ void __launch_bounds__(256) ctb_to_btc_add_kernel(const float* __restrict__ yin,
                                                             const float* __restrict__ skip,
                                                             const float* __restrict__ sa,
                                                             const float* __restrict__ sb,
                                                             float* __restrict__ out, int B, int C,
                                                             int T) {
  __shared__ float tl[64][33];
  const int tt = blockIdx.x, c = blockIdx.y, bt = blockIdx.z;
  const int t0 = tt * 32, b0 = bt * 64;
  for (int e = threadIdx.x; e < 64 * 32; e += 256) {
    const int tl_ = e / 64, bl = e % 64;
    const int b = b0 + bl, t = t0 + tl_;
    tl[bl][tl_] = (b < B && t < T) ? yin[((long long)c * T + t) * B + b] : 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 32; e += 256) {
    const int bl = e / 32, tl_ = e % 32;
    const int b = b0 + bl, t = t0 + tl_;
    if (b < B && t < T) {
      const long long i = ((long long)b * C + c) * T + t;
      const float v = tl[bl][tl_] + skip[i];
      out[i] = sa ? snake(v, sa[c], sb[c]) : v;
    }
  }
}

// nn.Tanh (codec_decoder.py:80) as a standalone module call (decoder.model run as the reference's
// nn.Sequential); inside decode() it is the last conv's epilogue (same tanhf).
__global__ void tanh_kernel(const float* __restrict__ x, float* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = tanhf(x[i]);
}

// Clip i, sample n: u = (splitmix64(0xB16C0DEC ^ (i<<32) ^ n) >> 40) * 2^-24, x = u - 0.5.
__global__ void synth_clips_kernel(float* __restrict__ x, int B, long long T, long long clip0) {
  const long long total = (long long)B * T;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const unsigned long long i = (unsigned long long)(clip0 + e / T);
    const unsigned long long n = (unsigned long long)(e % T);
    const unsigned long long h = splitmix64(0xB16C0DECull ^ (i << 32) ^ n);
    const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
    x[e] = u - 0.5f;
  }
}

static inline int grid_for(long long n, int block) {
  long long g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

int snake_launch(const float* x, const float* sa, const float* sb, float* y, int B, int C,
                 long long T, hipStream_t st) {
  const long long total = (long long)B * C * T;
  if (total == 0) return BC_OK;
  hipLaunchKernelGGL(snake_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, x, sa, sb, y, C, T,
                     total);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

// Streaming context window (streaming.py, causal streaming encode / decode): for each (b, c) row
//   win[j]     = j < P ? ctx[j] : act(x[j - P])   (j < P + n: the [carried context | chunk] input of a causal conv,
//                                                  or of a whole one-launch ResidualUnit)
//   ctx_out[i] = win[n + i]                        (i < P: the context the next chunk carries)
// in one pass.  act = SnakeBeta through snake() (bit-identical to snake_kernel's pairs and to the convs' Snake
// epilogue) or the identity; a missing ctx reads zeros (a stream's first chunk: the causal conv's zero padding,
// and snake(0) = 0, so zeros are the same before and after the activation).  x may be a strided view (row pitch
// xT, batch pitch xbs): a ResidualUnit run over its own window hands its last n columns on without a copy.
// 2-D grid (three 64-bit divisions per element): y walks the (b, c) rows (one 32-bit division per row),
// x the W = P + n window columns of a row
__global__ void __launch_bounds__(256) stream_window_kernel(const float* __restrict__ x, long long xbs, long long xT,
                                                            const float* __restrict__ ctx, const float* __restrict__ sa,
                                                            const float* __restrict__ sb, float* __restrict__ win,
                                                            float* __restrict__ ctx_out, int C, int n, int P, int rows) {
  const int W = P + n;
  for (int row = blockIdx.y; row < rows; row += gridDim.y) {
    const int b = row / C, c = row - b * C;
    const float* xr = x + (long long)b * xbs + (long long)c * xT;
    float* wr = win + (long long)row * W;
    const float a_ = sa ? sa[c] : 0.f, b_ = sa ? sb[c] : 0.f;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < W; j += gridDim.x * blockDim.x) {
      float v;
      if (j < P) {
        v = ctx ? ctx[(long long)row * P + j] : 0.f;
      } else {
        v = xr[j - P];
        if (sa) v = snake(v, a_, b_);
      }
      wr[j] = v;
      if (j >= n) ctx_out[(long long)row * P + (j - n)] = v;
    }
  }
}

int stream_window_launch(const float* x, long long xbs, long long xT, const float* ctx, const float* sa, const float* sb,
                         float* win, float* ctx_out, int B, int C, int n, int P, hipStream_t st) {
  if (!x || !win || B < 0 || C < 1 || n < 1 || P < 0 || xT < n || xbs < (long long)(C - 1) * xT + n) return BC_ERR_ARG;
  if ((sa == nullptr) != (sb == nullptr) || (P > 0 && !ctx_out)) return BC_ERR_ARG;
  const long long rows = (long long)B * C, W = (long long)P + n;
  if (rows == 0) return BC_OK;
  if (rows > 0x7fffffffLL || W > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  const int gx = (int)std::min<long long>((W + 255) / 256, 1024), gy = (int)std::min<long long>(rows, 65535);
  hipLaunchKernelGGL(stream_window_kernel, dim3(gx, gy), dim3(256), 0, st, x, xbs, xT, ctx, sa, sb, win, ctx_out, C, n,
                     P, (int)rows);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

// Activation1d with any (up_ratio, up taps, down_ratio, down taps) (act.py:8-23 constructor arguments):
// the same three stages as aa_snake_kernel, with the geometry of resample.py:10-33 / filter.py:86-95 at
// run time.  Up: replicate pad P = Ku / ru - 1, transposed conv stride ru, x ru, crop [PL, -PR) with
// PL = P ru + (Ku - ru) / 2; Snake; down: replicate pad (Kd / 2 - even, Kd / 2), conv stride rd.
// One workgroup = AA_TILE outputs of one (b, c) row; the tile's snake values s[j] (j = t rd + k - DL)
// and the x range they need sit in dynamic LDS.
__global__ void __launch_bounds__(256) aa_snake_gen_kernel(const float* __restrict__ x, const float* __restrict__ sa,
                                                           const float* __restrict__ sb, const float* __restrict__ fup,
                                                           const float* __restrict__ fdown, float* __restrict__ y,
                                                           int C, int T, int Tout, int ntiles, int ru, int ku, int rd,
                                                           int kd, int nx, int ns) {
  extern __shared__ float aa_sm[];
  float* fu = aa_sm;
  float* fd = fu + ku;
  float* xl = fd + kd;
  float* sl = xl + nx;
  const int tile = blockIdx.x % ntiles;
  const long long row = blockIdx.x / ntiles;  // b*C + c
  const int c = (int)(row % C);
  const float* xr = x + row * T;
  float* yr = y + row * (long long)Tout;
  const int t0 = tile * AA_TILE;
  const long long L = (long long)T * ru;            // up-sampled length
  const int up_pad = ku / ru - 1;
  const int up_pl = up_pad * ru + (ku - ru) / 2;    // crop offset into the transposed-conv output
  const int dn_pl = kd / 2 - (kd % 2 == 0 ? 1 : 0);
  for (int e = threadIdx.x; e < ku; e += 256) fu[e] = fup[e];
  for (int e = threadIdx.x; e < kd; e += 256) fd[e] = fdown[e];
  // s index range of the tile: j = t rd + k - dn_pl, clamped to [0, L) (replicate pad of the Snake output)
  const long long j0 = (long long)t0 * rd - dn_pl;
  const long long v0 = j0 < 0 ? 0 : (j0 >= L ? L - 1 : j0);
  // transposed-conv input indices i = (v + up_pl - k) / ru over the clamped v range
  const long long ibase = (v0 + up_pl - (ku - 1)) / ru - 1;
  for (int e = threadIdx.x; e < nx; e += 256) {
    long long xi = ibase + e - up_pad;  // padded index -> x index, replicate
    xi = xi < 0 ? 0 : (xi >= T ? T - 1 : xi);
    xl[e] = xr[xi];
  }
  __syncthreads();
  const float a = sa[c], ib = sb[c];
  const long long np = (long long)T + 2 * up_pad;  // padded input length
  for (int e = threadIdx.x; e < ns; e += 256) {
    long long v = j0 + e;
    v = v < 0 ? 0 : (v >= L ? L - 1 : v);
    const long long u = v + up_pl;
    float acc = 0.f;
    for (int k = (int)(u % ru); k < ku; k += ru) {  // out[u] = sum_{k: (u - k) % ru == 0} x_p[(u - k) / ru] f[k]
      const long long i = (u - k) / ru;
      if (i >= np) continue;
      if (i < 0) break;
      acc = acc + xl[i - ibase] * fu[k];
    }
    sl[e] = snake((float)ru * acc, a, ib);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < AA_TILE; e += 256) {
    const int t = t0 + e;
    if (t >= Tout) break;
    float acc = 0.f;
    for (int k = 0; k < kd; ++k) acc = acc + sl[e * rd + k] * fd[k];
    yr[t] = acc;
  }
}

// output length of the general activation (the down stage's conv over the padded up-sampled signal)
long long aa_snake_out_len(int T, int ru, int rd, int kd) {
  const long long L = (long long)T * ru;
  const int pl = kd / 2 - (kd % 2 == 0 ? 1 : 0), pr = kd / 2;
  const long long n = L + pl + pr - kd;
  return n < 0 ? 0 : n / rd + 1;
}

int aa_snake_gen_launch(const float* x, const float* sa, const float* sb, const float* fu, const float* fd, float* y,
                        int B, int C, int T, int ru, int ku, int rd, int kd, hipStream_t st) {
  if (ru < 1 || rd < 1 || ku < ru || kd < 1 || ku > 256 || kd > 256 || ru > 16 || rd > 16) return BC_ERR_UNSUPPORTED;
  const long long Tout = aa_snake_out_len(T, ru, rd, kd);
  if ((long long)B * C * T == 0 || Tout == 0) return BC_OK;
  if (Tout > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  const int ntiles = (int)((Tout + AA_TILE - 1) / AA_TILE);
  const long long nwg = (long long)B * C * ntiles;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  const int ns = (AA_TILE - 1) * rd + kd;
  const int nx = (ns + ku) / ru + 4;
  const size_t lds = (size_t)(ku + kd + nx + ns) * sizeof(float);
  if (lds > 64 * 1024) return BC_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(aa_snake_gen_kernel, dim3((unsigned)nwg), dim3(256), lds, st, x, sa, sb, fu, fd, y, C, T,
                     (int)Tout, ntiles, ru, ku, rd, kd, nx, ns);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int aa_snake_launch(const float* x, const float* sa, const float* sb, const float* fu,
                    const float* fd, float* y, int B, int C, int T, hipStream_t st) {
  if ((long long)B * C * T == 0) return BC_OK;
  const int ntiles = (T + AA_TILE - 1) / AA_TILE;
  const long long nwg = (long long)B * C * ntiles;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  hipLaunchKernelGGL(aa_snake_kernel, dim3((unsigned)nwg), dim3(256), 0, st, x, sa, sb, fu, fd, y, C,
                     T, ntiles);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int btc_to_ctb_launch(const float* x, float* y, int B, int C, int T, hipStream_t st) {
  if ((long long)B * C * T == 0) return BC_OK;
  dim3 grid((T + 31) / 32, C, (B + 63) / 64);
  hipLaunchKernelGGL(btc_to_ctb_kernel, grid, dim3(256), 0, st, x, y, B, C, T);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int ctb_to_btc_add_launch(const float* y, const float* skip, const float* sa, const float* sb,
                          float* out, int B, int C, int T, hipStream_t st) {
  if ((long long)B * C * T == 0) return BC_OK;
  dim3 grid((T + 31) / 32, C, (B + 63) / 64);
  hipLaunchKernelGGL(ctb_to_btc_add_kernel, grid, dim3(256), 0, st, y, skip, sa, sb, out, B, C, T);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

// [C][T][B] -> [C][T][B] with time reversed (the backward direction of a bidirectional LSTM runs the
// forward recurrence over the reversed sequence); B floats per (c, t) row, 16-byte moves when B % 4 == 0.
__global__ void time_reverse_kernel(const float* __restrict__ x, float* __restrict__ y, long long rows, int T, int B) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  if (B % 4 == 0) {
    const int q = B / 4;
    const long long n = rows * q;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
      const long long row = e / q, c = row / T;
      const int t = (int)(row - c * T), j = (int)(e - row * q);
      reinterpret_cast<float4*>(y)[(c * T + (T - 1 - t)) * q + j] = reinterpret_cast<const float4*>(x)[e];
    }
    return;
  }
  const long long n = rows * B;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += stride) {
    const long long row = e / B, c = row / T;
    const int t = (int)(row - c * T), b = (int)(e - row * B);
    y[(c * T + (T - 1 - t)) * B + b] = x[e];
  }
}

int time_reverse_launch(const float* x, float* y, int C, int T, int B, hipStream_t st) {
  const long long rows = (long long)C * T, n = rows * (B % 4 == 0 ? B / 4 : B);
  if (n == 0) return BC_OK;
  hipLaunchKernelGGL(time_reverse_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, x, y, rows, T, B);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int tanh_launch(const float* x, float* y, long long n, hipStream_t st) {
  if (n == 0) return BC_OK;
  hipLaunchKernelGGL(tanh_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, x, y, n);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int synth_clips_launch(float* x, int B, long long T, long long clip0, hipStream_t st) {
  const long long total = (long long)B * T;
  if (total == 0) return BC_OK;
  hipLaunchKernelGGL(synth_clips_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, x, B, T,
                     clip0);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

// ConvTranspose1d interleave (bc_convT1d_fwd_ws): output t of row (b, co) is phase r = (t + p) mod s, position
// q = (t + p) div s of that phase, i.e. element q - q_lo[r] of the phase's contiguous row (b, co) in the workspace.
// One thread per 4 consecutive outputs (16-byte stores where the row allows).
__global__ void __launch_bounds__(256) convT_interleave_kernel(const float* __restrict__ ph, const float* __restrict__ ph2,
                                                               float* __restrict__ y, float* __restrict__ y2, int Tout,
                                                               int Q4, long long plane, ConvTInterleave il, bool vec) {
  const long long row = blockIdx.y;  // b * Cout + co
  const int t0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (t0 >= Tout) return;
  float v[4], v2[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int t = t0 + k;
    if (t >= Tout) break;
    const int u = t + il.p;
    const int r = u % il.s, q = u / il.s;
    const long long src = r * plane + row * Q4 + (q - il.q_lo[r]);
    v[k] = ph[src];
    if (ph2) v2[k] = ph2[src];
  }
  float* yr = y + row * Tout;
  float* y2r = y2 ? y2 + row * Tout : nullptr;
  if (vec && t0 + 3 < Tout) {  // vec: Tout % 4 == 0 and y / y2 16-byte aligned (callers may pass views)
    *reinterpret_cast<floatx4*>(yr + t0) = floatx4{v[0], v[1], v[2], v[3]};
    if (y2r) *reinterpret_cast<floatx4*>(y2r + t0) = floatx4{v2[0], v2[1], v2[2], v2[3]};
  } else {
    for (int k = 0; k < 4 && t0 + k < Tout; ++k) {
      yr[t0 + k] = v[k];
      if (y2r) y2r[t0 + k] = v2[k];
    }
  }
}

int convT_interleave_launch(const float* ph, const float* ph2, float* y, float* y2, int B, int Cout, int Tout, int Q4,
                            const ConvTInterleave& il, hipStream_t st) {
  const long long rows = (long long)B * Cout;
  if (rows <= 0 || Tout <= 0) return BC_OK;
  if (rows > 65535 * 1024LL) return BC_ERR_UNSUPPORTED;
  const int gx = (Tout + 1023) / 1024;
  const bool vec = (Tout & 3) == 0 && (((unsigned long long)y | (unsigned long long)y2) & 15) == 0;
  // grid.y is limited to 65535: fold the rows into chunks
  for (long long r0 = 0; r0 < rows; r0 += 65535) {
    const int ny = (int)(rows - r0 < 65535 ? rows - r0 : 65535);
    hipLaunchKernelGGL(convT_interleave_kernel, dim3(gx, ny), dim3(256), 0, st, ph + r0 * Q4, ph2 ? ph2 + r0 * Q4 : nullptr,
                       y + r0 * Tout, y2 ? y2 + r0 * Tout : nullptr, Tout, Q4, (long long)rows * Q4, il, vec);
    BC_CHECK_LAUNCH();
  }
  return BC_OK;
}

}  // namespace bc
