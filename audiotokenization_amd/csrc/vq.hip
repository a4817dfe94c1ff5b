// Factorized VQ (vq/factorized_vector_quantize.py:29-108) for codebook_dim = 8.
//
//  vq_prepare_codebook_kernel : F.normalize(codebook) and codebook.pow(2).sum(1) (:99, :105).
//  vq_fwd_kernel              : per frame: in_proj (WN Linear D->8, :56) -> F.normalize (:98) ->
//                               dist = sum(e^2) - 2 e.c + sum(c^2) (:102-106) -> first argmin
//                               (== (-dist).max(1)[1], :107) -> z_q = codebook[idx] (:108) ->
//                               z_e + (z_q - z_e) (:68-70) -> out_proj (WN Linear 8->D, :72-74).
//  vq_argmin_kernel           : the search alone on given projected latents z_e.
//  vq2emb_kernel              : indices -> out_proj(codebook[idx]) (:78-91, residual_vq.py:42-48).
//  vq2emb_ct_kernel           : the token -> audio entry: stacked quantizers, (B, D, T) output.
//  fsq_fwd_kernel             : the FSQ quantizer (fsq=True decoders).
//  fsq_codes_kernel           : FSQ indices -> project_out(codes) (the fsq=True token -> latent step).
//
// Bit-exactness contract (tests/test_vq_*): given the same z_e, the indices equal the reference's.
// The fp32 operation order below restates what torch's CPU kernels do for these shapes, verified
// element-for-element in this container (oracle/vq_oracle.c header):
//   ||x||   = sqrt(((x0*x0 + x1*x1) + x2*x2) + ...)   sequential, separately rounded mul/add
//   e       = x / max(||x||, 1e-12)                    correctly rounded division
//   sum e^2 = sequential mul/add as above
//   e.c     = fma chain over k = 0..7 starting from 0 (MKL sgemm, K=8, >= 2 rows)
//   dist    = (sum_e2 - 2*dot) + sum_c2
// The library is built with -ffp-contract=off, so none of these are contracted.
#include "bc_common.h"
#include "bc_internal.h"

namespace bc {

constexpr int VQ_DIM = 8;

__device__ __forceinline__ void normalize8(float (&v)[VQ_DIM]) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < VQ_DIM; ++k) s = s + v[k] * v[k];
  float n = sqrtf(s);
  const float eps = 1e-12f;
  n = n < eps ? eps : n;  // clamp_min(eps); a NaN norm propagates as in torch's clamp_min
#pragma unroll
  for (int k = 0; k < VQ_DIM; ++k) v[k] = v[k] / n;
}

__device__ __forceinline__ float sumsq8(const float (&v)[VQ_DIM]) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < VQ_DIM; ++k) s = s + v[k] * v[k];
  return s;
}

__global__ void vq_prepare_codebook_kernel(const float* __restrict__ cb, float* __restrict__ cbn,
                                           float* __restrict__ csq, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v[VQ_DIM];
#pragma unroll
  for (int k = 0; k < VQ_DIM; ++k) v[k] = cb[(long long)i * VQ_DIM + k];
  normalize8(v);
#pragma unroll
  for (int k = 0; k < VQ_DIM; ++k) cbn[(long long)i * VQ_DIM + k] = v[k];
  csq[i] = sumsq8(v);
}

constexpr int VQ_CHUNK = 1024;  // codes staged per LDS pass (1024 * 9 floats = 36 KB)

// Search the whole codebook for one normalized row e (per lane); codes are staged into LDS in
// chunks and read by every lane at the same address (LDS broadcast).
__device__ __forceinline__ int vq_search(const float (&e)[VQ_DIM], float se,
                                         const float* __restrict__ cbn,
                                         const float* __restrict__ csq, int ncodes, float* lds_cb,
                                         float* lds_sq) {
  float best = __builtin_huge_valf();
  int bidx = 0;
  bool first = true;
  for (int c0 = 0; c0 < ncodes; c0 += VQ_CHUNK) {
    const int cn = min(VQ_CHUNK, ncodes - c0);
    __syncthreads();
    for (int q = threadIdx.x; q < cn * VQ_DIM; q += blockDim.x) lds_cb[q] = cbn[(long long)c0 * VQ_DIM + q];
    for (int q = threadIdx.x; q < cn; q += blockDim.x) lds_sq[q] = csq[c0 + q];
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < cn; ++k) {
      const float* c = lds_cb + k * VQ_DIM;
      float dot = 0.f;
#pragma unroll
      for (int q = 0; q < VQ_DIM; ++q) dot = fmaf(e[q], c[q], dot);
      const float dist = (se - 2.0f * dot) + lds_sq[k];
      // first index of the maximum of -dist: strict '<' keeps the earliest code on ties.  A NaN
      // distance never wins a comparison; torch's max() would propagate it, which cannot happen
      // for finite latents.
      if (first || dist < best) {
        best = dist;
        bidx = c0 + k;
        first = false;
      }
    }
  }
  return bidx;
}

// One thread per frame n = b*T + t.  z: [B][D][T]; outputs idx[B*T] (int64), optional
// z_e[B][8][T], optional post[B][D][T].
__global__ void __launch_bounds__(256) vq_fwd_kernel(
    const float* __restrict__ z, const float* __restrict__ w_in, const float* __restrict__ b_in,
    const float* __restrict__ cb, const float* __restrict__ cbn, const float* __restrict__ csq,
    const float* __restrict__ w_out, const float* __restrict__ b_out, long long* __restrict__ idx,
    float* __restrict__ ze_out, float* __restrict__ post, int B, int D, int T, int ncodes) {
  __shared__ float lds_cb[VQ_CHUNK * VQ_DIM];
  __shared__ float lds_sq[VQ_CHUNK];
  const long long NF = (long long)B * T;
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = n < NF;
  const long long nn = live ? n : NF - 1;
  const int b = (int)(nn / T), t = (int)(nn % T);
  const float* zb = z + (long long)b * D * T + t;

  // in_proj: z_e[j] = sum_d W[j][d] z[d] + bias[j]; the z column is loaded 16 channels at a time, so 16 loads are in
  // flight instead of one (one wave per SIMD here: each load's latency was exposed); the FMA chains keep d's order
  float ze[VQ_DIM];
#pragma unroll
  for (int q = 0; q < VQ_DIM; ++q) ze[q] = 0.f;
  constexpr int ZU = 16;
  int d = 0;
  for (; d + ZU <= D; d += ZU) {
    float zv[ZU];
#pragma unroll
    for (int j = 0; j < ZU; ++j) zv[j] = zb[(long long)(d + j) * T];
#pragma unroll
    for (int j = 0; j < ZU; ++j)
#pragma unroll
      for (int q = 0; q < VQ_DIM; ++q) ze[q] = fmaf(w_in[q * D + d + j], zv[j], ze[q]);
  }
  for (; d < D; ++d) {
    const float zv = zb[(long long)d * T];
#pragma unroll
    for (int q = 0; q < VQ_DIM; ++q) ze[q] = fmaf(w_in[q * D + d], zv, ze[q]);
  }
#pragma unroll
  for (int q = 0; q < VQ_DIM; ++q) ze[q] = ze[q] + b_in[q];
  if (ze_out && live)
#pragma unroll
    for (int q = 0; q < VQ_DIM; ++q) ze_out[((long long)b * VQ_DIM + q) * T + t] = ze[q];

  float e[VQ_DIM];
#pragma unroll
  for (int q = 0; q < VQ_DIM; ++q) e[q] = ze[q];
  normalize8(e);
  const float se = sumsq8(e);
  const int k = vq_search(e, se, cbn, csq, ncodes, lds_cb, lds_sq);
  if (!live) return;
  idx[n] = k;
  if (post) {
    float st[VQ_DIM];
#pragma unroll
    for (int q = 0; q < VQ_DIM; ++q) {
      const float zq = cb[(long long)k * VQ_DIM + q];
      st[q] = ze[q] + (zq - ze[q]);  // straight-through, forward value
    }
    float* pb = post + (long long)b * D * T + t;
    for (int d = 0; d < D; ++d) {
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < VQ_DIM; ++q) acc = fmaf(w_out[d * VQ_DIM + q], st[q], acc);
      pb[(long long)d * T] = acc + b_out[d];
    }
  }
}

// z_e rows [N][8] -> idx[N]
__global__ void __launch_bounds__(256) vq_argmin_kernel(const float* __restrict__ ze,
                                                        const float* __restrict__ cbn,
                                                        const float* __restrict__ csq,
                                                        long long* __restrict__ idx, long long N,
                                                        int ncodes) {
  __shared__ float lds_cb[VQ_CHUNK * VQ_DIM];
  __shared__ float lds_sq[VQ_CHUNK];
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nn = n < N ? n : N - 1;
  float e[VQ_DIM];
#pragma unroll
  for (int q = 0; q < VQ_DIM; ++q) e[q] = ze[nn * VQ_DIM + q];
  normalize8(e);
  const float se = sumsq8(e);
  const int k = vq_search(e, se, cbn, csq, ncodes, lds_cb, lds_sq);
  if (n < N) idx[n] = k;
}

// emb[n][d] = b_out[d] + sum_q W_out[d][q] * cb[idx[n]][q]     (output (N, D), as vq2emb returns)
__global__ void vq2emb_kernel(const long long* __restrict__ idx, long long idx_stride,
                              const float* __restrict__ cb, const float* __restrict__ w_out,
                              const float* __restrict__ b_out, float* __restrict__ emb, long long N,
                              int D, int accumulate) {
  const long long total = N * D;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const long long n = e / D;
    const int d = (int)(e % D);
    const long long k = idx[n * idx_stride];
    float v;
    if (w_out) {
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < VQ_DIM; ++q) acc = fmaf(w_out[d * VQ_DIM + q], cb[k * VQ_DIM + q], acc);
      v = acc + b_out[d];
    } else {
      v = cb[k * VQ_DIM + d];  // proj=False: embed_code only
    }
    emb[e] = accumulate ? emb[e] + v : v;
  }
}

// FSQ quantizer (decoder fsq=True, codec_decoder.py:41-47, 85-92 -> the vendored lucidrains
// finite_scalar_quantization.py FSQ.forward, eval, channel_first, one codebook).  One thread per frame:
//   zi[j]   = project_in: fma chain over the D channels from 0, + bias[j]        (nn.Linear D -> d)
//   b[j]    = tanh(zi[j] + shift[j]) * half_l[j] - offset[j]                        (bound, :118-123)
//   q[j]    = b[j] + (rint(b[j]) - b[j])                  (round_ste's forward value; rint = half to even)
//   code[j] = q[j] / half_width[j]                                                  (quantize, :147-149)
//   idx     = int( sum_j (code[j] * half_width[j] + half_width[j]) * basis[j] )     (codes_to_indices)
//   post[b][c][t] = fma chain over j of w_out[c][j] * code[j] from 0, + b_out[c]   (project_out)
// The per-level constants are computed on the host with the reference's own float32 torch expressions
// (modules.FSQ.constants) and passed as consts[5][d] = half_l, offset, shift, half_width, basis.
constexpr int FSQ_MAXD = 8;
__global__ void __launch_bounds__(256) fsq_fwd_kernel(const float* __restrict__ z, const float* __restrict__ w_in,
                                                      const float* __restrict__ b_in, const float* __restrict__ w_out,
                                                      const float* __restrict__ b_out, const float* __restrict__ consts,
                                                      int* __restrict__ idx, float* __restrict__ post, int B, int D,
                                                      int T, int nd) {
  const long long NF = (long long)B * T;
  const long long n = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= NF) return;
  const int b = (int)(n / T), t = (int)(n % T);
  const float* zb = z + (long long)b * D * T + t;
  float zi[FSQ_MAXD];
#pragma unroll
  for (int j = 0; j < FSQ_MAXD; ++j) zi[j] = 0.f;
  for (int c = 0; c < D; ++c) {
    const float zv = zb[(long long)c * T];
#pragma unroll
    for (int j = 0; j < FSQ_MAXD; ++j)
      if (j < nd) zi[j] = fmaf(w_in[j * D + c], zv, zi[j]);
  }
  float code[FSQ_MAXD];
  float isum = 0.f;
#pragma unroll
  for (int j = 0; j < FSQ_MAXD; ++j) {
    if (j >= nd) {
      code[j] = 0.f;
      continue;
    }
    const float half_l = consts[j], offset = consts[nd + j], shift = consts[2 * nd + j];
    const float hw = consts[3 * nd + j], basis = consts[4 * nd + j];
    const float v = zi[j] + b_in[j];
    const float bd = tanhf(v + shift) * half_l - offset;
    const float q = bd + (rintf(bd) - bd);
    code[j] = q / hw;
    isum = isum + (code[j] * hw + hw) * basis;
  }
  idx[n] = (int)isum;
  if (post) {
    float* pb = post + (long long)b * D * T + t;
    for (int c = 0; c < D; ++c) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < FSQ_MAXD; ++j)
        if (j < nd) acc = fmaf(w_out[c * nd + j], code[j], acc);
      pb[(long long)c * T] = acc + b_out[c];
    }
  }
}

int fsq_fwd_launch(const float* z, const float* w_in, const float* b_in, const float* w_out, const float* b_out,
                   const float* consts, int* idx, float* post, int B, int D, int T, int nd, hipStream_t st) {
  if (!z || !w_in || !b_in || !consts || !idx || B < 0 || D < 1 || T < 0 || nd < 1) return BC_ERR_ARG;
  if ((post != nullptr) != (w_out != nullptr) || (w_out != nullptr) != (b_out != nullptr)) return BC_ERR_ARG;
  if (nd > FSQ_MAXD) return BC_ERR_UNSUPPORTED;
  const long long NF = (long long)B * T;
  if (NF == 0) return BC_OK;
  const long long nwg = (NF + 255) / 256;
  if (nwg > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(fsq_fwd_kernel, dim3((unsigned)nwg), dim3(256), 0, st, z, w_in, b_in, w_out, b_out, consts, idx,
                     post, B, D, T, nd);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

// FSQ token -> latent (finite_scalar_quantization.py:159-192 indices_to_codes, channel_first, one codebook; the
// fsq=True decoder's inverse of forward's indices): idx[B][T] (int32 or int64) -> post[B][D][T] = project_out(codes).
//   lvl[j]  = floor(idx / basis[j]) mod levels[j]  (torch's // and % on integers: floor division, non-negative
//             modulo, so any integer maps to a grid point exactly as the reference maps it, :170-174)
//   code[j] = float(lvl[j] - hw[j]) / float(hw[j])  (_scale_and_shift_inverse, :155-157: integer difference,
//             true division in fp32)
//   post    = fsq_fwd_kernel's project_out chain (fma over j from 0, + b_out), so an index forward produced
//             decodes to forward's own post bit for bit (its q is the integer lvl - hw).
// Thread = one position t, the workgroup walks FSQ_CT_D channels (stores coalesced along t).
constexpr int FSQ_CT_D = 32;
struct FsqLevels {
  long long basis[FSQ_MAXD];
  int levels[FSQ_MAXD];
};
__global__ void __launch_bounds__(256) fsq_codes_kernel(const void* __restrict__ idx, int idx64, FsqLevels lv, int nd,
                                                        const float* __restrict__ w_out, const float* __restrict__ b_out,
                                                        float* __restrict__ post, int T, int D) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int d0 = blockIdx.y * FSQ_CT_D;
  const int b = blockIdx.z;
  if (t >= T) return;
  const long long n = (long long)b * T + t;
  const long long k = idx64 ? static_cast<const long long*>(idx)[n] : (long long)static_cast<const int*>(idx)[n];
  float code[FSQ_MAXD];
#pragma unroll
  for (int j = 0; j < FSQ_MAXD; ++j) {
    code[j] = 0.f;
    if (j < nd) {
      const long long bs = lv.basis[j], L = lv.levels[j];
      long long qd = k / bs;
      if ((k % bs != 0) && ((k < 0) != (bs < 0))) --qd;  // floor division
      long long m = qd % L;
      if (m < 0) m += L;                                   // floor modulo (L > 0)
      const long long hw = L / 2;
      code[j] = (float)(m - hw) / (float)hw;
    }
  }
  float* out = post + ((long long)b * D + d0) * T + t;
  const int dn = D - d0 < FSQ_CT_D ? D - d0 : FSQ_CT_D;
  for (int dd = 0; dd < dn; ++dd) {
    const int c = d0 + dd;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < FSQ_MAXD; ++j)
      if (j < nd) acc = fmaf(w_out[c * nd + j], code[j], acc);
    out[(long long)dd * T] = acc + b_out[c];
  }
}

int fsq_codes_launch(const void* idx, int idx_bits, const int* levels, const float* w_out, const float* b_out,
                     float* post, int B, int D, int T, int nd, hipStream_t st) {
  if (!idx || !levels || !w_out || !b_out || !post || B < 0 || D < 1 || T < 0 || nd < 1) return BC_ERR_ARG;
  if (idx_bits != 32 && idx_bits != 64) return BC_ERR_ARG;
  if (nd > FSQ_MAXD) return BC_ERR_UNSUPPORTED;
  FsqLevels lv{};
  long long basis = 1;
  for (int j = 0; j < nd; ++j) {
    if (levels[j] < 2) return BC_ERR_ARG;  // hw = levels // 2 divides
    lv.levels[j] = levels[j];
    lv.basis[j] = basis;                   // cumprod([1] + levels[:-1]) (:76-77)
    basis *= levels[j];
    if (basis > (1LL << 40)) return BC_ERR_UNSUPPORTED;
  }
  if (B == 0 || T == 0) return BC_OK;
  if (B > 65535 || (D + FSQ_CT_D - 1) / FSQ_CT_D > 65535) return BC_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(fsq_codes_kernel, dim3((T + 255) / 256, (D + FSQ_CT_D - 1) / FSQ_CT_D, B), dim3(256), 0, st, idx,
                     idx_bits == 64 ? 1 : 0, lv, nd, w_out, b_out, post, T, D);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

// Token -> audio entry (codec_decoder.py:96-99 -> residual_vq.py:42-48 -> factorized_vector_quantize.py:78-81,
// then the caller's transpose(1, 2)): idx[B][T][Nq] -> emb[B][D][T], the decoder's input layout, so the
// transpose costs nothing.  Per quantizer q: v = (fma chain over k of w_out_q[d][k] * cb_q[idx][k] from 0) +
// b_out_q[d], exactly vq2emb_kernel's order; the sum over quantizers starts from 0. as the reference's
// `quantized_out = 0.` does.  Parameters of the Nq quantizers are stacked: cb [Nq][n_codes][8],
// w_out [Nq][D][8], b_out [Nq][D].  An index outside [0, n_codes) yields NaN for its column (no
// out-of-range read).  Thread = one position t; the workgroup walks VQ_CT_D channels, so the
// stores are coalesced along t and the weights are wave-uniform (scalar loads).
constexpr int VQ_CT_D = 32;
constexpr int VQ_CT_MAXQ = 8;
__global__ void __launch_bounds__(256) vq2emb_ct_kernel(const long long* __restrict__ idx, int nq,
                                                        const float* __restrict__ cb, const float* __restrict__ w_out,
                                                        const float* __restrict__ b_out, float* __restrict__ emb,
                                                        int T, int D, int n_codes) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int d0 = blockIdx.y * VQ_CT_D;
  const int b = blockIdx.z;
  if (t >= T) return;
  float c[VQ_CT_MAXQ][VQ_DIM];
  bool bad = false;
  for (int q = 0; q < nq; ++q) {
    const long long k = idx[((long long)b * T + t) * nq + q];
    const bool ok = k >= 0 && k < n_codes;
    bad = bad || !ok;
    const float* row = cb + ((long long)q * n_codes + (ok ? k : 0)) * VQ_DIM;
#pragma unroll
    for (int j = 0; j < VQ_DIM; ++j) c[q][j] = row[j];
  }
  float* out = emb + ((long long)b * D + d0) * T + t;
  const int dn = D - d0 < VQ_CT_D ? D - d0 : VQ_CT_D;
  for (int dd = 0; dd < dn; ++dd) {
    const int d = d0 + dd;
    float sum = 0.f;
    for (int q = 0; q < nq; ++q) {
      const float* w = w_out + ((long long)q * D + d) * VQ_DIM;
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < VQ_DIM; ++j) acc = fmaf(w[j], c[q][j], acc);
      sum = sum + (acc + b_out[(long long)q * D + d]);
    }
    out[(long long)dd * T] = bad ? __builtin_nanf("") : sum;
  }
}

int vq2emb_ct_launch(const long long* idx, int nq, const float* cb, const float* w_out, const float* b_out,
                     float* emb, int B, int T, int D, int n_codes, hipStream_t st) {
  if (nq < 1 || nq > VQ_CT_MAXQ || B < 0 || T < 0 || D < 1 || n_codes < 1 || !idx || !cb || !w_out || !b_out ||
      !emb)
    return BC_ERR_ARG;
  if (B == 0 || T == 0) return BC_OK;
  if (B > 65535 || (D + VQ_CT_D - 1) / VQ_CT_D > 65535) return BC_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(vq2emb_ct_kernel, dim3((T + 255) / 256, (D + VQ_CT_D - 1) / VQ_CT_D, B), dim3(256), 0, st,
                     idx, nq, cb, w_out, b_out, emb, T, D, n_codes);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

// ResidualVQ bookkeeping (residual_vq.py:31-33): residual -= q; out += q
__global__ void rvq_update_kernel(float* __restrict__ residual, float* __restrict__ out,
                                  const float* __restrict__ q, long long n, int first) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float qi = q[i];
    residual[i] = residual[i] - qi;
    out[i] = first ? 0.f + qi : out[i] + qi;
  }
}

static inline int grid_for(long long n, int block) {
  long long g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

int vq_prepare_launch(const float* cb, float* cbn, float* csq, int n, hipStream_t st) {
  if (n <= 0) return BC_ERR_ARG;
  hipLaunchKernelGGL(vq_prepare_codebook_kernel, dim3((n + 255) / 256), dim3(256), 0, st, cb, cbn,
                     csq, n);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int vq_fwd_launch(const float* z, const float* w_in, const float* b_in, const float* cb,
                  const float* cbn, const float* csq, const float* w_out, const float* b_out,
                  long long* idx, float* ze_out, float* post, int B, int D, int T, int ncodes,
                  hipStream_t st) {
  const long long NF = (long long)B * T;
  if (NF == 0) return BC_OK;
  const long long nwg = (NF + 255) / 256;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  hipLaunchKernelGGL(vq_fwd_kernel, dim3((unsigned)nwg), dim3(256), 0, st, z, w_in, b_in, cb, cbn,
                     csq, w_out, b_out, idx, ze_out, post, B, D, T, ncodes);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int vq_argmin_launch(const float* ze, const float* cbn, const float* csq, long long* idx,
                     long long N, int ncodes, hipStream_t st) {
  if (N == 0) return BC_OK;
  const long long nwg = (N + 255) / 256;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  hipLaunchKernelGGL(vq_argmin_kernel, dim3((unsigned)nwg), dim3(256), 0, st, ze, cbn, csq, idx, N,
                     ncodes);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int vq2emb_launch(const long long* idx, long long idx_stride, const float* cb, const float* w_out,
                  const float* b_out, float* emb, long long N, int D, int accumulate,
                  hipStream_t st) {
  const long long total = N * D;
  if (total == 0) return BC_OK;
  hipLaunchKernelGGL(vq2emb_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st, idx, idx_stride, cb,
                     w_out, b_out, emb, N, D, accumulate);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int rvq_update_launch(float* residual, float* out, const float* q, long long n, int first,
                      hipStream_t st) {
  if (n == 0) return BC_OK;
  hipLaunchKernelGGL(rvq_update_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, residual, out, q,
                     n, first);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

}  // namespace bc
