// A whole ResidualUnit (vq/module.py:74-89) at C = 192 in ONE launch on the 16-wave 192 x 256 conv tile (x6):
//   y = x + conv1( snake2( conv7_d( snake1(x) ) ) )
// followed by the unit's epilogue (bias, residual, optional next Snake, dual output).
//
// Two launches (k=7 conv, then the k=1 conv) move h = snake2(conv7(...)) through HBM: written once, read once, plus
// the pointwise launch's own staging and barriers -- 27 ms per config-2 step over the nine C >= 192 units (VERDICT r05
// item 1).  At C = 192 one 192-row tile covers every channel, so the workgroup that finishes the k=7 conv of a
// 256-column block holds all of h for it:
//   phase 1: conv1d_x6_body, exactly the standalone k=7 launch's main loop (16-byte input staging, LDS-DMA weight
//            copies, one tap per K-step), with the weights as the MFMA A operand (!SWAP) so a lane ends with four
//            consecutive channels of one column; optional snake1 on load (SIN);
//   phase 2: the block in two halves of 128 columns (a half = n-tile j of every wave; 144 KiB of LDS):
//            bridge  -- h = snake2(acc + b7), split exactly into 3 bf16 planes, written to LDS as the k=1 conv's input
//                       tile Hs[plane][32-ch chunk][128 cols][64 B] (16-B groups XOR-swizzled by column, the layout of
//                       resunit_x6.hip's bridge); h never leaves the CU;
//            k=1     -- each wave computes 3 m-tiles x 2 n-tiles (48 rows x 32 columns of the half) over K = 192 with
//                       h as the MFMA A operand (transposed tile: the shared 16-byte epilogue) and the k=1 weight
//                       fragments loaded from global memory into registers (4 waves read each fragment; the 216 KiB of
//                       split k=1 weights do not fit beside Hs);
//            epilogue -- conv_epilogue.h: + b1, + x (residual), next Snake / dual output.
//   Half 1's bridge runs while the other waves finish half 0's epilogue (barrier between the k=1 reads of half 0
//   and the Hs writes of half 1).
// Same weight packing as bc_conv1d_pack for cfg 122 (one m-group: M = C = 192).
#include <cstdio>
#include <cstdlib>

#include "bc_common.h"
#include "bc_internal.h"
#include "conv1d_x6_kernel.h"
#include "conv_epilogue.h"
#include "x6_common.h"

namespace bc {

struct RUW16Args {
  const float* w1;   // packed k=1 weights (cfg 122: [chunk][plane][m-tile][lane][8 bf16])
  const float* s2a;  // Snake between the two convs: alpha_exp [C]
  const float* s2b;  //                               inv_beta  [C]
};

constexpr int W16_C = 192;                  // channels (one 192-row m-group)
constexpr int W16_QA = 12;                  // m-tiles
constexpr int W16_NCK = W16_C / X6_BKC;     // 32-channel chunks of the k=1 input
constexpr int W16_HC = 128;                 // columns per half
constexpr int W16_HPLANE = W16_NCK * W16_HC * 64;  // bytes per Hs plane (48 KiB)
constexpr int W16_MAXD = 9;                 // the B staging covers the k7 halo at dilation <= 9
constexpr int W16_COEF = 3 * W16_HPLANE;    // LDS: per-channel coefficients [6][192] floats (b7, s2a, s2b, b1, osa, osb), past
                                            // every phase-1 buffer (x6_lds <= 131.5 KiB at d <= 9) and Hs
constexpr int W16_LDS_EXTRA = 8 * W16_C * 4;  // + [6] isa, [7] isb (snake on load, SIN 2)

// (16-B groups XOR-swizzled by (n >> 2) & 3: the phase-2 fragment reads are 2-way conflicted, the bridge's 8-byte
// writes 2-way under any 16-B swizzle; the conflict-free (n >> 1) & 3 halved the conflict cycles and changed no unit's
// time, profiles/r06s_hs_swizzle_rejected.txt)
__device__ __forceinline__ int w16_hs_off(int n, int g) { return n * 64 + 16 * (g ^ ((n >> 2) & 3)); }

// SIN: 2 = snake on load with the coefficients staged in LDS (0 = the producer activated x)
// B4: the 16-byte input staging (Tin % 4 == 0, 16-B aligned rows: every encoder shape); else single-float loads
// P: 3 = x6 (three exact bf16 planes, six products; phase 1 one tap per K-step, as the x6 k7 launches), 1 = the bf16
// precision mode of config 5 (one plane, one product; phase 1 four taps per K-step over two B buffers, as the bf16 k7
// launches; h rounded to bf16 where the pointwise conv's staging rounded it)
template <int P, int SIN, bool B4>
__global__ void __launch_bounds__(1024, 1) resunit_w16_kernel(ConvArgs a, ConvArgs e, RUW16Args r) {
  static_assert(P == 3 || P == 1, "x6 or bf16 operands");
  typedef bf16x8_t frag_t;
  constexpr int TPS1 = P == 3 ? 1 : 4;  // phase-1 taps per K-step
  constexpr bool DB1 = P == 1;          // phase-1 double-buffered B tile
  {  // the per-channel coefficients into LDS by LDS-DMA (landed by the body's prologue vmcnt(0) + barrier):
     // [0] b7, [1] s2a, [2] s2b (bridge), [3] b1, [4] osa, [5] osb (epilogue; zeros when absent)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (int q = wave; q < (SIN ? 24 : 18); q += 16) {
      const int k = q / 3, part = q % 3;
      const float* src = k == 0 ? a.bias : k == 1 ? r.s2a : k == 2 ? r.s2b : k == 3 ? e.bias : k == 4 ? e.osa
                         : k == 5 ? e.osb : k == 6 ? a.isa : a.isb;
      unsigned char* dst = smem_xb + W16_COEF + k * (W16_C * 4) + part * 256;
      if (src)
        __builtin_amdgcn_global_load_lds((const void*)(src + part * 64 + lane), (lds_void_t)dst, 4, 0, 0);
      else
        reinterpret_cast<float*>(dst)[lane] = 0.f;
    }
  }
  conv1d_x6_body<6, 2, 2, 8, P, false, TPS1, DB1, B4, false, SIN>(
      a, [&](floatx4 (&acc)[6][2], int b, int m0, int n0, int wm, int wn, int lane, float) {
        (void)m0;
        unsigned char* Hs = smem_xb;  // aliases the phase-1 B tile and A buffers: every wave has passed the last
                                      // K-step's barrier and no copy is in flight (the last step issued none)
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int mg = wave & 3, ng = wave >> 2;  // phase 2: rows 48 mg .. + 48, local n-tiles 2 ng, 2 ng + 1

        // bridge of half j: this wave's n-tile j (6 m-tiles x 16 columns) -> Hs
        auto bridge = [&](int j) {
          const int n = wn * 16 + (lane & 15);  // local column
#pragma unroll
          for (int i = 0; i < 6; ++i) {
            const int co = wm * 96 + i * 16 + (lane >> 4) * 4;  // 4 consecutive channels co..co+3
            const float* cf = reinterpret_cast<const float*>(smem_xb + W16_COEF) + co;
            const floatx4 bias = *reinterpret_cast<const floatx4*>(cf);
            const floatx4 sa = *reinterpret_cast<const floatx4*>(cf + W16_C);
            const floatx4 sb = *reinterpret_cast<const floatx4*>(cf + 2 * W16_C);
            const f32x2 lo = snake_pk((f32x2){acc[i][j][0] + bias[0], acc[i][j][1] + bias[1]}, (f32x2){sa[0], sa[1]},
                                      (f32x2){sb[0], sb[1]});
            const f32x2 hi = snake_pk((f32x2){acc[i][j][2] + bias[2], acc[i][j][3] + bias[3]}, (f32x2){sa[2], sa[3]},
                                      (f32x2){sb[2], sb[3]});
            unsigned char* dst = Hs + (co / X6_BKC) * (W16_HC * 64) + w16_hs_off(n, (co % X6_BKC) / 8) + (co % 8) * 2;
            if constexpr (P == 1) {  // h rounded to bf16 (the pointwise conv's staging rounding)
              *reinterpret_cast<u32x2_t*>(dst) = (u32x2_t){pk_bf16(lo.x, lo.y), pk_bf16(hi.x, hi.y)};
              continue;
            }
            unsigned h0, m0_, l0, h1, m1, l1;
            split2(lo.x, lo.y, h0, m0_, l0);
            split2(hi.x, hi.y, h1, m1, l1);
            *reinterpret_cast<u32x2_t*>(dst) = (u32x2_t){h0, h1};
            *reinterpret_cast<u32x2_t*>(dst + W16_HPLANE) = (u32x2_t){m0_, m1};
            *reinterpret_cast<u32x2_t*>(dst + 2 * W16_HPLANE) = (u32x2_t){l0, l1};
          }
        };

        // the k=1 conv over Hs: acc2[i][jj] = rows 48 mg + 16 i, local columns (2 ng + jj) * 16 ..
        const unsigned char* w1b = reinterpret_cast<const unsigned char*>(r.w1) + lane * 16;
        auto wfrag = [&](int kc, int i, frag_t (&w)[P]) {
#pragma unroll
          for (int p = 0; p < P; ++p)
            w[p] = *reinterpret_cast<const frag_t*>(w1b + ((kc * P + p) * W16_QA + mg * 3 + i) * 1024);
        };
        auto phase2 = [&](floatx4 (&acc2)[3][2]) {
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) acc2[i][jj] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
          for (int kc = 0; kc < W16_NCK; ++kc) {
            frag_t hf[2][P];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const unsigned char* src = Hs + kc * (W16_HC * 64) + w16_hs_off((2 * ng + jj) * 16 + (lane & 15), lane >> 4);
#pragma unroll
              for (int p = 0; p < P; ++p) hf[jj][p] = *reinterpret_cast<const frag_t*>(src + p * W16_HPLANE);
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) {
              // (loaded at the m-tile that uses it: a prefetch one m-tile ahead spilled 37 VGPRs; the other three
              // waves of the SIMD cover the L1 / L2 latency)
              frag_t w[P];
              if (BC_ABL(e.dbg, 2)) {
#pragma unroll
                for (int p = 0; p < P; ++p) w[p] = hf[p & 1][0];
              } else {
                wfrag(kc, i, w);
              }
              if (BC_ABL(e.dbg, 1)) {
                acc2[i][0][0] += (float)w[0][0] + (float)w[P - 1][1];
                continue;
              }
#pragma unroll
              for (int jj = 0; jj < 2; ++jj) {
                floatx4 t = acc2[i][jj];
                if constexpr (P == 1) {  // one bf16 product (h as A: the transposed tile of the shared epilogue)
                  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[jj][0], w[0], t, 0, 0, 0);
                } else {
                  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[jj][0], w[2], t, 0, 0, 0);
                  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[jj][1], w[1], t, 0, 0, 0);
                  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[jj][2], w[0], t, 0, 0, 0);
                  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[jj][0], w[1], t, 0, 0, 0);
                  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[jj][1], w[0], t, 0, 0, 0);
                  t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(hf[jj][0], w[0], t, 0, 0, 0);
                }
                acc2[i][jj] = t;
              }
            }
          }
        };
        // epilogue of half j: the residual's 16-byte groups are loaded early (load_res, in flight across a barrier and
        // a bridge, or under phase 2's MFMAs); coefficients from LDS; conv_epilogue.h's per-element operation order
        const float* rb = e.res + (long long)b * e.rbs;
        float* yb = e.y + (long long)b * e.ybs;
        float* y2b = e.y2 ? e.y2 + (long long)b * e.ybs : nullptr;
        const bool snk = e.osa != nullptr;
        auto ncol0 = [&](int jj, int j) { return n0 + (2 * ng + jj) * 32 + j * 16 + (lane >> 4) * 4; };
        auto load_res = [&](int j, floatx4 (&rr)[3][2]) {
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const int co = mg * 48 + i * 16 + (lane & 15), nb = ncol0(jj, j);
              rr[i][jj] = floatx4{0.f, 0.f, 0.f, 0.f};
              if (e.vec && nb + 3 < e.Nout && BC_DOK((long long)co * e.yT + nb + 3 < e.rbs))
                rr[i][jj] = *reinterpret_cast<const floatx4*>(rb + (long long)co * e.yT + nb);
            }
        };
        auto epilogue = [&](const floatx4 (&acc2)[3][2], const floatx4 (&rr)[3][2], int j) {
          if (BC_ABL(e.dbg, 4)) {
            if (acc2[0][0][0] == 1234.5f && rr[0][0][0] == 1.f) e.y[0] = 0.f;  // keep the work alive
            return;
          }
          const float* cf = reinterpret_cast<const float*>(smem_xb + W16_COEF);
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const int co = mg * 48 + i * 16 + (lane & 15);
            const float bias = cf[3 * W16_C + co], sa = cf[4 * W16_C + co], sb = cf[5 * W16_C + co];
            const long long rowoff = (long long)co * e.yT;
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const int nb = ncol0(jj, j);
              if (nb >= e.Nout) continue;
              if (e.vec && nb + 3 < e.Nout) {
                const long long yi = rowoff + nb;
                if (!BC_DOK(yi >= 0 && yi + 3 < e.ybs)) continue;
                floatx4 v, sv;
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = rr[i][jj][q] + (acc2[i][jj][q] + bias);
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
              } else {  // a partial group at the clip's end (or a launch without 16-byte accesses)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  const int nn = nb + q;
                  if (nn >= e.Nout) break;
                  const long long yi = rowoff + nn;
                  if (!BC_DOK(yi >= 0 && yi < e.ybs && yi < e.rbs)) break;
                  const float v = rb[yi] + (acc2[i][jj][q] + bias);
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
        };

        floatx4 acc2[3][2], rr[3][2];
        if (BC_ABL(e.dbg, 8)) {
          if (acc[0][0][0] == 1234.5f && acc[5][1][3] == 1.f) Hs[0] = 1;
        } else {
          bridge(0);
        }
        lds_barrier();
        phase2(acc2);
        load_res(0, rr);
        lds_barrier();  // every wave is done reading half 0's Hs
        if (BC_ABL(e.dbg, 8)) {
          if (acc[0][1][0] == 1234.5f) Hs[0] = 1;
        } else {
          bridge(1);
        }
        epilogue(acc2, rr, 0);
        lds_barrier();
        load_res(1, rr);
        phase2(acc2);
        epilogue(acc2, rr, 1);
      });
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
// BC_RU_W16=0 keeps the C = 192 units on two launches (A/B timing).
static bool ru_w16_on() {
  static const bool v = [] {
    const char* e = getenv("BC_RU_W16");
    return !e || atoi(e) != 0;
  }();
  return v;
}

static size_t w16_lds(int d, int P) {
  const X6Tile t{6, 2, 2, 8};
  // B tile(s) + double-buffered A: x6 one tap per K-step, bf16 four taps over two B buffers (the k7 launches' variants)
  const size_t ph1 = P == 3 ? x6_lds(t, x6_ncol(t, 7, 1, d), 3, 1) : x6_lds(t, x6_ncol(t, 7, 1, d), 1, 1, 4, 2);
  if (ph1 > (size_t)W16_COEF) return ~(size_t)0;             // the coefficients sit past phase 1's buffers
  return (size_t)W16_COEF + W16_LDS_EXTRA;
}

bool resunit_w16_ok(int C, int d, int P) {
  return ru_w16_on() && (P == 3 || P == 1) && C == W16_C && d >= 1 && d <= W16_MAXD && w16_lds(d, P) <= 160 * 1024;
}

int resunit_w16_launch(ConvArgs& a, ConvArgs& e, const float* w1, const float* s2a, const float* s2b, int B, int P,
                       hipStream_t st) {
  if (P != 3 && P != 1) return BC_ERR_ARG;
  if (a.Cin != W16_C || a.Cout != W16_C || a.K != 7 || a.s != 1 || a.d < 1 || a.d > W16_MAXD) return BC_ERR_UNSUPPORTED;
  const X6Tile t{6, 2, 2, 8};
  const int ncol = x6_ncol(t, 7, 1, a.d);
  if (ncol > 32 * X6_MAXCOL_ITERS) return BC_ERR_UNSUPPORTED;
  a.ps = 0;
  a.ntm = 1;
  a.ntn = (a.Nout + 255) / 256;
  a.nchunks = W16_NCK;
  a.win = ncol;
  a.bpitch = x6_pitch(1);
  a.bstage = (ncol * a.bpitch + 15) / 16 * 16;
  a.wsc = nullptr;
  a.prio = 0;
  const long long nwg = (long long)a.ntn * B;
  if (nwg <= 0) return BC_OK;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  if ((long long)a.Cin * a.Tin * 4 > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  a.nwg = (int)nwg;
  const size_t lds = w16_lds(a.d, P);
  if (lds > 160 * 1024) return BC_ERR_UNSUPPORTED;
  RUW16Args r{w1, s2a, s2b};
  // BC_W16_DEBUG (BC_ABLATION builds only, wrong results, timing): 1 no phase-2 MFMAs, 2 no k=1 weight loads, 4 no
  // epilogue, 8 no bridge; BC_X6_DEBUG: the phase-1 main loop's switches (conv1d_x6_kernel.h)
  static const int dbg2 = [] {
    const char* v = getenv("BC_W16_DEBUG");
    return v ? atoi(v) : 0;
  }();
  static const int dbg1 = [] {
    const char* v = getenv("BC_X6_DEBUG");
    return v ? atoi(v) : 0;
  }();
  e.dbg = dbg2;
  a.dbg = dbg1;
  const bool b4 = x6_b4_on() && x6_b4_fits(a);
  a.sin_lds = W16_COEF + 6 * W16_C * 4;
#define BC_W16_LAUNCH(PP)                                                                                    \
  if (a.isa && b4)                                                                                           \
    hipLaunchKernelGGL((resunit_w16_kernel<PP, 2, true>), dim3(a.nwg), dim3(1024), lds, st, a, e, r);        \
  else if (a.isa)                                                                                            \
    hipLaunchKernelGGL((resunit_w16_kernel<PP, 2, false>), dim3(a.nwg), dim3(1024), lds, st, a, e, r);       \
  else if (b4)                                                                                               \
    hipLaunchKernelGGL((resunit_w16_kernel<PP, 0, true>), dim3(a.nwg), dim3(1024), lds, st, a, e, r);        \
  else                                                                                                       \
    hipLaunchKernelGGL((resunit_w16_kernel<PP, 0, false>), dim3(a.nwg), dim3(1024), lds, st, a, e, r);
  if (P == 3) {
    BC_W16_LAUNCH(3)
  } else {
    BC_W16_LAUNCH(1)
  }
#undef BC_W16_LAUNCH
  BC_CHECK_LAUNCH();
  return BC_OK;
}

}  // namespace bc

BC_DEBUG_EXPORT(resunit_w16)
