/*
 * vq_oracle.c — plain-C restatement of FactorizedVectorQuantize.decode_latents
 * (BigCodec_SSL/vq/factorized_vector_quantize.py:93-108) — TEST INFRASTRUCTURE ONLY.
 * Only tests/ (and the smoke check) load this; the product never does.
 *
 * The fp32 operation order restates what torch 2.10 CPU kernels do for these shapes (established
 * element-for-element against torch in the development container; pinned by
 * tests/golden/vq_decode_latents.npz, which the reference itself produced):
 *   F.normalize (:98-99):   n = sqrt(((x0*x0 + x1*x1) + x2*x2) + ...)  (mul and add each rounded)
 *                           x / max(n, 1e-12)                          (IEEE division)
 *   pow(2).sum(1) (:103,105): same sequential mul/add
 *   encodings @ codebook.t() (:104): MKL sgemm with K = 8 is an fma chain k = 0..7 from 0
 *                           (for >= 2 rows; a single row takes MKL's GEMV path instead)
 *   dist = (se - 2*dot) + sc; indices = (-dist).max(1)[1]  -> first minimum (:107)
 * Build: gcc -O2 -ffp-contract=off -fPIC -shared (oracle/build.py); no -ffast-math.
 */
#include <math.h>
#include <stdint.h>

#define DIM 8

static void normalize8(const float* in, float* out) {
  float s = 0.f;
  for (int k = 0; k < DIM; ++k) {
    float p = in[k] * in[k];
    s = s + p;
  }
  float n = sqrtf(s);
  const float eps = 1e-12f;
  if (n < eps) n = eps;
  for (int k = 0; k < DIM; ++k) out[k] = in[k] / n;
}

static float sumsq8(const float* v) {
  float s = 0.f;
  for (int k = 0; k < DIM; ++k) {
    float p = v[k] * v[k];
    s = s + p;
  }
  return s;
}

/* codebook [n_codes][8] raw -> normalized [n_codes][8] and sum of squares [n_codes] */
void vq_oracle_prepare(const float* cb, float* cbn, float* csq, int n_codes) {
  for (int i = 0; i < n_codes; ++i) {
    normalize8(cb + (int64_t)i * DIM, cbn + (int64_t)i * DIM);
    csq[i] = sumsq8(cbn + (int64_t)i * DIM);
  }
}

/* z_e rows [n][8] -> idx [n]; also writes the winning distance and the runner-up distance (fp32) */
void vq_oracle_argmin(const float* ze, const float* cbn, const float* csq, int64_t n, int n_codes,
                      int64_t* idx, float* best_out, float* second_out) {
  for (int64_t r = 0; r < n; ++r) {
    float e[DIM];
    normalize8(ze + r * DIM, e);
    const float se = sumsq8(e);
    float best = INFINITY, second = INFINITY;
    int bi = 0, first = 1;
    for (int k = 0; k < n_codes; ++k) {
      const float* c = cbn + (int64_t)k * DIM;
      float dot = 0.f;
      for (int q = 0; q < DIM; ++q) dot = fmaf(e[q], c[q], dot);
      const float dist = (se - 2.0f * dot) + csq[k];
      if (first || dist < best) {
        second = best;
        best = dist;
        bi = k;
        first = 0;
      } else if (dist < second) {
        second = dist;
      }
    }
    idx[r] = bi;
    if (best_out) best_out[r] = best;
    if (second_out) second_out[r] = second;
  }
}
