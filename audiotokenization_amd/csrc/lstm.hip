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
