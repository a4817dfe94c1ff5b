// ResLSTM recurrence (vq/module.py:143-167 -> torch.nn.LSTM, batch_first, unidirectional).
//
// Layout: the sequence lives in "ctb" layout [H][T*B] (element (j, t, b) at j*T*B + t*B + b), so
//   * the input projection of every timestep is ONE conv1d k=1 GEMM over a single "clip" of length
//     T*B (conv1d.hip, M = 4H, K = H, N = T*B), including b_ih + b_hh;
//   * step t reads its 64 batch columns of each gate row as contiguous 256-B runs;
//   * a layer's output is already the next layer's input layout.
// One launch per timestep: each workgroup owns J = 4 hidden units (16 gate rows: gate-major i,f,g,o
// as torch orders them) and 64 batch columns; its 4 waves split K = H four ways and reduce through
// LDS, then 256 threads apply the cell update  c = f*c + i*g,  h = o*tanh(c).
#include "bc_common.h"
#include "bc_internal.h"

namespace bc {

constexpr int LSTM_J = 4;

// whh_p: [H/J][H/4 ksteps][64 lanes]; lane -> (m = lane&15 -> gate m>>2, unit m&3; k = 4ks + lane>>4)
__global__ void __launch_bounds__(256) lstm_step_kernel(const float* __restrict__ gx,
                                                        const float* __restrict__ whh_p,
                                                        float* __restrict__ y,
                                                        float* __restrict__ cst, int H, int B,
                                                        int T, int t) {
  __shared__ float red[4][16][68];
  const int ug = blockIdx.x;
  const int bc0 = blockIdx.y * 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long TB = (long long)T * B;
  const int j0 = ug * LSTM_J;

  if (t > 0) {
    floatx4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int kq = H / 4;            // k values per wave
    const int ks0 = w * (kq / 4);    // first k-step of this wave
    const int nks = kq / 4;
    const float* ap = whh_p + ((long long)ug * (H / 4) + ks0) * 64 + lane;
    const float* hp = y + (long long)(t - 1) * B;
    const int bl = lane & 15;
    for (int ks = 0; ks < nks; ++ks) {
      const float av = ap[(long long)ks * 64];
      const int k = (ks0 + ks) * 4 + (lane >> 4);
      const float* hrow = hp + (long long)k * TB;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int b = bc0 + nt * 16 + bl;
        const float bv = b < B ? hrow[b] : 0.f;
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[nt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][(lane >> 4) * 4 + r][nt * 16 + (lane & 15)] = acc[nt][r];
  }
  __syncthreads();
  const int jj = tid >> 6;   // unit within group
  const int bl = tid & 63;
  const int b = bc0 + bl;
  if (b >= B) return;
  const int j = j0 + jj;
  if (j >= H) return;
  float g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v = gx[((long long)q * H + j) * TB + (long long)t * B + b];
    if (t > 0) {
      const int m = q * 4 + jj;
      const float hsum = ((red[0][m][bl] + red[1][m][bl]) + red[2][m][bl]) + red[3][m][bl];
      v = v + hsum;
    }
    g[q] = v;
  }
  const float ig = sigmoidf_ref(g[0]);
  const float fg = sigmoidf_ref(g[1]);
  const float gg = tanhf(g[2]);
  const float og = sigmoidf_ref(g[3]);
  const long long ci = (long long)j * B + b;
  const float cprev = t > 0 ? cst[ci] : 0.f;
  const float c = fg * cprev + ig * gg;
  cst[ci] = c;
  y[(long long)j * TB + (long long)t * B + b] = og * tanhf(c);
}

// ------------------------------------------------------------------------------------------------
// Fast step kernel (H % 128 == 0): 8 waves split K; each wave holds its W_hh slice in registers
// (NKW k-steps, loaded as float4) and streams h_{t-1} from a fragment-native buffer:
//   hfrag[cg][ks][lane][nt] = h[4ks + (lane>>4)][64cg + 16nt + (lane&15)]
// so every k-step is ONE 16-byte load per lane (1 KiB per wave-instruction).  The producer of step
// t writes its 4 units x 64 batch columns as one contiguous 1 KiB block of that layout.
// whh_p2: [H/J][8 waves][NKW/4][64 lanes][4]  (k = 4*(w*NKW + 4q + i) + (lane>>4))
// ------------------------------------------------------------------------------------------------
constexpr int LSTM_W = 8;

template <int NKW>
__global__ void __launch_bounds__(512) lstm_step_frag_kernel(const float* __restrict__ gx,
                                                             const float* __restrict__ whh_p2,
                                                             const float* __restrict__ hin,
                                                             float* __restrict__ hout,
                                                             float* __restrict__ y,
                                                             float* __restrict__ cst, int H, int B,
                                                             int T, int t) {
  __shared__ float red[LSTM_W][16][68];
  const int ug = blockIdx.x;
  const int cg = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const long long TB = (long long)T * B;
  if (t > 0) {
    const floatx4* ap = reinterpret_cast<const floatx4*>(whh_p2) +
                        ((long long)(ug * LSTM_W + w) * (NKW / 4)) * 64 + lane;
    floatx4 a[NKW / 4];
#pragma unroll
    for (int q = 0; q < NKW / 4; ++q) a[q] = ap[q * 64];
    const floatx4* hp = reinterpret_cast<const floatx4*>(hin) +
                        ((long long)cg * (H / 4) + (long long)w * NKW) * 64 + lane;
    floatx4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NKW; ++ks) {
      const floatx4 bv = hp[ks * 64];
      const float av = a[ks >> 2][ks & 3];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[nt], acc[nt], 0, 0, 0);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w][(lane >> 4) * 4 + r][nt * 16 + (lane & 15)] = acc[nt][r];
  }
  __syncthreads();
  if (tid >= 256) return;
  const int jj = tid >> 6;  // unit within the group of 4
  const int bl = tid & 63;
  const int b = cg * 64 + bl;
  const int j = ug * LSTM_J + jj;
  float g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v = b < B ? gx[((long long)q * H + j) * TB + (long long)t * B + b] : 0.f;
    if (t > 0) {
      const int m = q * 4 + jj;
      float hsum = red[0][m][bl];
#pragma unroll
      for (int ww = 1; ww < LSTM_W; ++ww) hsum = hsum + red[ww][m][bl];
      v = v + hsum;
    }
    g[q] = v;
  }
  const float ig = sigmoidf_ref(g[0]);
  const float fg = sigmoidf_ref(g[1]);
  const float gg = tanhf(g[2]);
  const float og = sigmoidf_ref(g[3]);
  float h = 0.f;
  if (b < B) {
    const long long ci = (long long)j * B + b;
    const float cprev = t > 0 ? cst[ci] : 0.f;
    const float c = fg * cprev + ig * gg;
    cst[ci] = c;
    h = og * tanhf(c);
    y[(long long)j * TB + (long long)t * B + b] = h;
  }
  // fragment-native copy of h_t for the next step: [cg][ks = ug][lane = jj*16 + (bl&15)][nt = bl>>4]
  hout[(((long long)cg * (H / 4) + ug) * 64 + jj * 16 + (bl & 15)) * 4 + (bl >> 4)] = h;
}

void lstm_pack_hh2(const float* w, float* out, int H) {
  const int nkw = H / 4 / LSTM_W;
  long long o = 0;
  for (int ug = 0; ug < H / LSTM_J; ++ug)
    for (int wv = 0; wv < LSTM_W; ++wv)
      for (int q = 0; q < nkw / 4; ++q)
        for (int lane = 0; lane < 64; ++lane)
          for (int i = 0; i < 4; ++i, ++o) {
            const int m = lane & 15;
            const int row = (m >> 2) * H + ug * LSTM_J + (m & 3);
            const int k = 4 * (wv * nkw + 4 * q + i) + (lane >> 4);
            out[o] = w[(long long)row * H + k];
          }
}

bool lstm_fast_ok(int H) {
  const int nkw = H / 4 / LSTM_W;
  return H % 128 == 0 && (nkw == 4 || nkw == 8 || nkw == 16 || nkw == 32 || nkw == 48);
}

int lstm_step_frag_launch(const float* gx, const float* whh_p2, const float* hin, float* hout,
                          float* y, float* cst, int H, int B, int T, int t, hipStream_t st) {
  dim3 grid(H / LSTM_J, (B + 63) / 64);
  const int nkw = H / 4 / LSTM_W;
#define BC_LSTM_CASE(N)                                                                           \
  case N:                                                                                         \
    hipLaunchKernelGGL(lstm_step_frag_kernel<N>, grid, dim3(512), 0, st, gx, whh_p2, hin, hout, y, \
                       cst, H, B, T, t);                                                          \
    break;
  switch (nkw) {
    BC_LSTM_CASE(4)
    BC_LSTM_CASE(8)
    BC_LSTM_CASE(16)
    BC_LSTM_CASE(32)
    BC_LSTM_CASE(48)
    default:
      return BC_ERR_UNSUPPORTED;
  }
#undef BC_LSTM_CASE
  BC_CHECK_LAUNCH();
  return BC_OK;
}

void lstm_pack_hh(const float* w, float* out, int H) {
  // w: [4H][H] row-major (torch weight_hh_l{k}: rows i,f,g,o)
  long long o = 0;
  for (int ug = 0; ug < H / LSTM_J; ++ug)
    for (int ks = 0; ks < H / 4; ++ks)
      for (int lane = 0; lane < 64; ++lane, ++o) {
        const int m = lane & 15;
        const int row = (m >> 2) * H + ug * LSTM_J + (m & 3);
        const int k = ks * 4 + (lane >> 4);
        out[o] = w[(long long)row * H + k];
      }
}

int lstm_step_launch(const float* gx, const float* whh_p, float* y, float* cst, int H, int B, int T,
                     int t, hipStream_t st) {
  dim3 grid(H / LSTM_J, (B + 63) / 64);
  hipLaunchKernelGGL(lstm_step_kernel, grid, dim3(256), 0, st, gx, whh_p, y, cst, H, B, T, t);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

}  // namespace bc
