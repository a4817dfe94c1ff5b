// Shared epilogue of the conv kernels (conv1d.hip fp32 MFMA, conv1d_x6.hip 3xbf16 MFMA).
//
// Both kernels issue their MFMAs with the operands swapped (input fragment as "A", weight fragment
// as "B"), which computes the TRANSPOSED output tile: in the 16x16 C/D layout a lane then holds
// four CONSECUTIVE output positions of ONE output channel,
//   co = tile_row0 + (lane & 15),   n = tile_col0 + (lane >> 4) * 4 + r   (r = 0..3),
// so the epilogue reads the residual and writes the outputs as one 16-byte access per lane and
// tile (4x fewer store instructions than a channel-per-register layout, the store-issue bound of a
// k=1 conv's epilogue), and fetches bias / Snake coefficients once per channel.
// Op order per element is the reference's: (acc + bias), residual + that, then tanh or Snake.
#pragma once
#include "bc_common.h"
#include "bc_internal.h"

namespace bc {

__device__ __forceinline__ float conv_epi_value(const ConvArgs& a, float acc, float bias, float res,
                                                bool has_res) {
  float v = acc + bias;
  if (has_res) v = res + v;
  if (a.epi == 1) v = tanhf(v);
  return v;
}

// acc[i][j]: transposed 16x16 tiles; rows (channels) start at row0 + 16 i, columns (positions) at
// col0 + 16 j.
// SC (h3 kernels): the accumulator holds x*S_x times w*S_w[co] products; acc * (a.wsc[co] * xinv)
// (a power of two: exact) restores the fp32 dot product before the bias is added.
// RP / rpre (MT == 1 only): the residual's 16-byte groups already loaded by the caller, one per n-tile,
// for exactly the lanes / tiles that take the 16-byte path (conv_epilogue_res).
// Loads run in passes of RPS m-tiles (all MT where the registers allow, else 2), each pass's per-row coefficients
// and residual groups issued before its first store: vmcnt retires in issue order and counts stores, so a bias or
// residual load issued behind m-tile i's stores can only be waited for once those stores have completed -- with a
// load per m-tile that was one dependent store round trip per m-tile (6 per tile on the 192-row tiles, now 2).
// RPSX: the pass size forced by the caller (0: the rule above; 1 where the two-m-tile passes' registers spill, e.g. the
// h3 multi-tap 16-wave kernels: 7 -> 41 spilled VGPRs, the phase-decomposed strided launch 22 -> 31 ms per step,
// profiles/r05r_ab_h3.txt)
template <int MT, int NT, bool SC, bool RP, int RPSX = 0>
__device__ __forceinline__ void conv_epilogue_impl(const ConvArgs& a, const floatx4 (&acc)[MT][NT], int b, int row0,
                                                   int col0, int lane, float xinv, const floatx4 (&rpre)[NT]) {
  float* yb = a.y + (long long)b * a.ybs;
  float* y2b = a.y2 ? a.y2 + (long long)b * a.ybs : nullptr;
  const float* rb = a.res ? a.res + (long long)b * a.rbs : nullptr;
  const bool snk = a.osa != nullptr;
  auto vec_tile = [&](int co, int nb) { return co < a.Cout && a.vec && nb + 3 < a.Nout; };
  constexpr int RPS = (MT == 1 && RP) ? 1 : RPSX ? RPSX : (MT * NT <= 8 ? MT : 2);
  float pbias[RPS], psa[RPS], psb[RPS], psc[RPS];
  auto load_p = [&](int i, int k) {
    const int co = row0 + i * 16 + (lane & 15);
    const bool ok = co < a.Cout;
    pbias[k] = ok && a.bias ? a.bias[co] : 0.f;
    psa[k] = ok && snk ? a.osa[co] : 0.f;
    psb[k] = ok && snk ? a.osb[co] : 0.f;
    psc[k] = SC && ok ? a.wsc[co] * xinv : 1.f;
  };
  floatx4 rr[RPS][NT];
  auto load_r = [&](int i, floatx4 (&d)[NT]) {
    const int co = row0 + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int nb = col0 + j * 16 + (lane >> 4) * 4;
      d[j] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (rb && vec_tile(co, nb) && BC_DOK(co >= 0 && nb >= 0 && (long long)co * a.yT + a.ooff + nb + 3 < a.rbs))
        d[j] = *reinterpret_cast<const floatx4*>(rb + (long long)co * a.yT + a.ooff + nb);
    }
  };
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    if (i % RPS == 0) {  // the pass's coefficients and residual groups, before its first store
#pragma unroll
      for (int k = 0; k < RPS; ++k)
        if (i + k < MT) {
          load_p(i + k, k);
          if (!(MT == 1 && RP)) load_r(i + k, rr[k]);
        }
    }
    const int co = row0 + i * 16 + (lane & 15);
    if (co >= a.Cout) continue;
    const float bias = pbias[i % RPS];
    const float sa = psa[i % RPS];
    const float sb = psb[i % RPS];
    const float sc = psc[i % RPS];
    const long long rowoff = (long long)co * a.yT + a.ooff;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int nb = col0 + j * 16 + (lane >> 4) * 4;
      if (nb >= a.Nout) continue;
      if (vec_tile(co, nb)) {
        const long long yi = rowoff + nb;
        if (!BC_DOK(yi >= 0 && yi + 3 < a.ybs)) continue;  // debug build: the tile's 16 bytes inside the batch item
        const floatx4 r = (MT == 1 && RP) ? rpre[j] : rr[i % RPS][j];
        floatx4 v, sv;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          v[q] = conv_epi_value(a, SC ? acc[i][j][q] * sc : acc[i][j][q], bias, r[q], rb != nullptr);
        if (snk) {
          const f32x2 lo = snake_pk((f32x2){v[0], v[1]}, splat2(sa), splat2(sb));
          const f32x2 hi = snake_pk((f32x2){v[2], v[3]}, splat2(sa), splat2(sb));
          sv = (floatx4){lo.x, lo.y, hi.x, hi.y};
        } else {
          sv = v;
        }
        if (y2b) {
          *reinterpret_cast<floatx4*>(yb + yi) = v;
          *reinterpret_cast<floatx4*>(y2b + yi) = sv;
        } else {
          *reinterpret_cast<floatx4*>(yb + yi) = sv;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = nb + q;
          if (n >= a.Nout) break;
          const long long yi = rowoff + (long long)n * a.ostride;
          if (!BC_DOK(yi >= 0 && yi < a.ybs && (!rb || yi < a.rbs))) break;
          const float v =
              conv_epi_value(a, SC ? acc[i][j][q] * sc : acc[i][j][q], bias, rb ? rb[yi] : 0.f, rb != nullptr);
          if (snk) {
            const float sv = snake(v, sa, sb);
            if (y2b) {
              yb[yi] = v;
              y2b[yi] = sv;
            } else {
              yb[yi] = sv;
            }
          } else {
            yb[yi] = v;
          }
        }
      }
    }
  }
}

template <int MT, int NT, bool SC = false, int RPSX = 0>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, const floatx4 (&acc)[MT][NT], int b, int row0,
                                              int col0, int lane, float xinv = 1.f) {
  conv_epilogue_impl<MT, NT, SC, false, RPSX>(a, acc, b, row0, col0, lane, xinv, acc[0]);
}
template <int NT, bool SC = false>
__device__ __forceinline__ void conv_epilogue_res(const ConvArgs& a, const floatx4 (&acc)[1][NT], int b, int row0,
                                                  int col0, int lane, float xinv, const floatx4 (&rpre)[NT]) {
  conv_epilogue_impl<1, NT, SC, true>(a, acc, b, row0, col0, lane, xinv, rpre);
}

// Host: may the epilogue use 16-byte accesses for this launch?  (unit output stride, every row
// and batch offset a multiple of 4 floats, 16-byte aligned base pointers)
inline int conv_epilogue_vec_ok(const ConvArgs& a) {
  auto al = [](const void* p) { return ((unsigned long long)p & 15ull) == 0; };
  if (a.ostride != 1 || a.yT % 4 || a.ooff % 4 || a.ybs % 4) return 0;
  if (!al(a.y) || (a.y2 && !al(a.y2))) return 0;
  if (a.res && (a.rbs % 4 || !al(a.res))) return 0;
  return 1;
}

}  // namespace bc
