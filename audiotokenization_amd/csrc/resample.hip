// Band-limited sinc resampling (the real-audio ingest of extract_indices.py:129-132 and
// data_module.py:95-98: torchaudio.transforms.Resample(orig_freq, new_freq), default
// sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99).
//
// torchaudio's _apply_sinc_resample_kernel pads the signal by (width, width + orig) zeros, runs
// conv1d(stride = orig) with `new` filters of K = 2 * width + orig taps, interleaves the `new` output
// phases and keeps ceil(new * L / orig) samples.  Restated per output sample o = j * new + k:
//   y[o] = sum_{m < K} kern[k][m] * x[j * orig + m - width]      (x = 0 outside [0, L))
// with the filters built on the host exactly as torchaudio does (ingest.sinc_resample_kernel: float64
// arithmetic, cast to float32).  The sum runs in tap order with fused multiply-adds.
//
// One thread per output sample; the workgroup stages its filters (new x K floats, <= 128 KiB) in LDS
// (larger filter banks are read through L1 / L2).
// Consecutive threads read consecutive input samples (stride orig / new per thread): coalesced,
// HBM-bound (4 B in + 4 B out per sample at 16 -> 24 kHz).  Rows of y have a pitch >= Lout so the
// caller can leave extract_indices.py:135-137's pad_to_stride zeros behind each row.
#include "bc_common.h"
#include "bc_internal.h"

namespace bc {

constexpr int RS_BLOCK = 256;
constexpr int RS_MAX_KERN = 32768;  // floats of filter staged in LDS (128 KiB)

// LDSW: filters staged in LDS (nw * K <= RS_MAX_KERN), else read through the caches (e.g. 22050 ->
// 24000 Hz: 160 phases x 161 taps).
template <bool LDSW>
__global__ void __launch_bounds__(RS_BLOCK) resample_sinc_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                 const float* __restrict__ kern, long long Lin,
                                                                 long long Lout, long long ypitch, int orig, int nw,
                                                                 int K, int width) {
  extern __shared__ float kl[];
  if (LDSW) {
    for (int i = threadIdx.x; i < nw * K; i += RS_BLOCK) kl[i] = kern[i];
    __syncthreads();
  }
  const int b = blockIdx.y;
  const long long o = (long long)blockIdx.x * RS_BLOCK + threadIdx.x;
  if (o >= Lout) return;
  const long long j = o / nw;
  const int k = (int)(o - j * nw);
  const long long s = j * orig - width;
  const float* xb = x + (long long)b * Lin;
  const float* w = (LDSW ? kl : kern) + k * K;
  float acc = 0.f;
  if (s >= 0 && s + K <= Lin) {
    for (int m = 0; m < K; ++m) acc = fmaf(w[m], xb[s + m], acc);
  } else {
    for (int m = 0; m < K; ++m) {
      const long long t = s + m;
      const float v = (t >= 0 && t < Lin) ? xb[t] : 0.f;
      acc = fmaf(w[m], v, acc);
    }
  }
  y[(long long)b * ypitch + o] = acc;
}

int resample_sinc_launch(const float* x, float* y, const float* kern, int B, long long Lin, long long Lout,
                         long long ypitch, int orig, int nw, int K, int width, hipStream_t st) {
  if (!x || !y || !kern || B < 0 || Lin < 0 || Lout < 0 || ypitch < Lout || orig < 1 || nw < 1 || K < 1 ||
      width < 0)
    return BC_ERR_ARG;
  if (B > 65535) return BC_ERR_UNSUPPORTED;
  if (B == 0 || Lout == 0) return BC_OK;
  const long long nblk = (Lout + RS_BLOCK - 1) / RS_BLOCK;
  if (nblk > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  if ((long long)nw * K <= RS_MAX_KERN)
    hipLaunchKernelGGL(resample_sinc_kernel<true>, dim3((unsigned)nblk, B), dim3(RS_BLOCK), (size_t)nw * K * 4, st, x,
                       y, kern, Lin, Lout, ypitch, orig, nw, K, width);
  else
    hipLaunchKernelGGL(resample_sinc_kernel<false>, dim3((unsigned)nblk, B), dim3(RS_BLOCK), 0, st, x, y, kern, Lin,
                       Lout, ypitch, orig, nw, K, width);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

}  // namespace bc
