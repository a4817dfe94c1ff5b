// A whole ResidualUnit (vq/module.py:74-89) in ONE launch, fp32-accurate 3xbf16 MFMA:
//   y = x + conv1( snake2( conv7_d( x_act ) ) )      (x_act = snake1(x), produced upstream)
// followed by the same epilogue as a lone conv (bias, residual, optional next Snake, dual output).
//
// Unfused, a ResidualUnit is two launches and the k=7 conv's activated output h (C x T) makes a full
// HBM round trip; at C <= 192 the k=1 conv is a short-K GEMM whose epilogue and staging dominate.
// Here one workgroup owns ALL C channels of a BN-column tile:
//   phase 1: the k=7 conv exactly as conv1d_x6_kernel's main loop (weights as the MFMA A operand, so
//            a lane ends with 4 consecutive channels of one column);
//   bridge : h = acc + b7, snake2, exact 3-plane bf16 split, written to LDS as the k=1 conv's input
//            tile Hs[plane][32-ch chunk][col][32 ch] (64-B rows, 16-B groups XOR-swizzled by col so
//            the 16 columns of a ds_read_b128 quarter-wave hit disjoint banks) - h never leaves LDS;
//   phase 2: the k=1 conv over Hs (input as the MFMA A operand: transposed tile for the shared
//            16-byte epilogue, conv_epilogue.h).  Each wave owns one m-tile and a group of n-tiles and
//            holds that m-tile's k=1 weights in registers (C <= 128: at most 48 VGPRs), so phase 2
//            needs no weight copies and no barrier, and Hs may reuse the whole phase-1 LDS
//            (Bs + As): a 96 x 128 tile fits in 80 KiB, i.e. two workgroups per CU.
// Same weight packing as bc_conv1d_pack for the unit's cfg (M = C in a single m-group).
// P = 3: x6 (3 bf16 planes, 6 products); P = 2: h3 (2 block-scaled fp16 planes, 3 products; the k=7
// input is scaled per staged chunk as in conv1d_x6.hip, h per workgroup tile from its block maximum);
// P = 1: bf16 (one plane, one product: the bf16 precision mode, x and h rounded to bf16 like the lone
// bf16 convs round their inputs).
#include <cstdio>
#include <cstdlib>

#include "bc_common.h"
#include "bc_internal.h"
#include "conv_epilogue.h"
#include "x6_common.h"

namespace bc {

constexpr int RU_MAX_DIL = 9;  // the B loads are sized for the k7 halo at dilation <= 9 (BigCodec: 1, 3, 9)

struct RUExtra {
  const float* w1;   // packed k=1 weights
  const float* s2a;  // Snake between the two convs: alpha_exp [C]
  const float* s2b;  //                               inv_beta  [C]
  int hplane;        // bytes per Hs plane = nck1 * BN * 64
  int nck1;          // 32-channel chunks of the k=1 conv's input
  int dbg;           // BC_RU_DEBUG timing experiments (wrong results, BC_ABLATION builds only): 1 no A copies, 2 no B
                     // loads, 4 no epilogue, 8 no phase 2, 16 no Snake on load, 32 no phase-1 MFMAs, 64 no bridge Snake
  // snake on load: the unit's first Activation1d applied while staging the k=7 input (x_act == x_raw,
  // isa / isb = its alpha_exp / inv_beta), so the producer writes only the raw tensor; nullptr: x_act given
  const float* isa;
  const float* isb;
};

// (16-B groups XOR-swizzled by (n >> 2) & 3: the phase-2 fragment reads are 2-way conflicted, the bridge's 8-byte
// writes 2-way under any 16-B swizzle; the conflict-free (n >> 1) & 3 halved the conflict cycles and changed no unit's
// time, profiles/r06s_hs_swizzle_rejected.txt)
__device__ __forceinline__ int hs_off(int n, int g) { return n * 64 + 16 * (g ^ ((n >> 2) & 3)); }

// Minimum waves per SIMD the unit is compiled for: 4 (<= 128 VGPRs, two workgroups per CU) for the NT = 1
// tiles and the 48 x 32-per-wave C = 96 tile (123); 2 otherwise (the 48 x 512 tile 124 spills 234 VGPRs at 128:
// its phase 2 holds 16 n-tiles per wave).
constexpr int ru_min_waves(int MT, int NT, int WM, int P) {
  return (NT == 1 || (MT == 3 && NT == 2 && WM == 2)) ? 4 : 2;
}
// 16-wave tiles (1024 threads, one workgroup per CU, four waves per SIMD: <= 128 VGPRs) declare 1, as the conv kernel
constexpr int ru_launch_waves(int MT, int NT, int WM, int WN, int P) {
  return WM * WN == 16 ? 1 : ru_min_waves(MT, NT, WM, P);
}
// phase 2 (k=1 conv): QA m-tiles x NTT n-tiles over the NW waves, NPW n-tile groups per m-tile (the largest divisor of
// NTT within NW / QA)
constexpr int ru_npw(int NW, int QA, int NTT) {
  int n = NW / QA < NTT ? NW / QA : NTT;
  while (n > 1 && NTT % n) --n;
  return n;
}

// TPS: k=7 taps per phase-1 K-step (one A copy, one wait and one barrier per TPS taps).
template <int MT, int NT, int WM, int WN, int P, int TPS = 1>
__global__ void __launch_bounds__(64 * WM * WN, ru_launch_waves(MT, NT, WM, WN, P)) resunit_x6_kernel(ConvArgs a, ConvArgs e, RUExtra r) {
  static_assert(P >= 1 && P <= 3, "bf16, h3 or x6 operands");
  typedef typename FragType<P>::type frag_t;
  constexpr int NW = WM * WN;  // 8 waves (512 threads, two workgroups per CU) or 16 (1024, one per CU)
  static_assert(NW == 8 || NW == 16, "512- or 1024-thread workgroups");
  constexpr int NTHR = 64 * NW;
  constexpr int NCG = NW / 8;  // B staging column groups (16 channel pairs x 32 column lanes each)
  __shared__ unsigned smax[2][NW];  // P == 2: per-wave block maxima (k=7 input chunks by parity; h tile)
  constexpr int BN = 16 * NT * WN;
  constexpr int QA = WM * MT;
  constexpr int CI = ((BN + 6 * RU_MAX_DIL + 31) / 32 + NCG - 1) / NCG;  // 32-column B passes per thread
  // phase 2 (k=1 conv): QA m-tiles x NTT n-tiles over the NW waves, NPW n-tile groups per m-tile
  constexpr int NTT = NT * WN;
  static_assert(QA <= NW, "one m-tile per wave in phase 2");
  constexpr int NPW = ru_npw(NW, QA, NTT);
  constexpr int NTW = NTT / NPW;
  static_assert(NTT % NPW == 0, "n-tile groups");
  constexpr int KC1 = (16 * QA + X6_BKC - 1) / X6_BKC;  // k=1 input chunks (C = 16 * QA)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_ru[];

  const int ncol = a.win;
  const int bplane = a.bstage;
  unsigned char* Bs = smem_ru;                 // phase 1: [P][ncol][64 B] (16-B groups swizzled, x6_pitch)
  unsigned char* As = smem_ru + P * bplane;    // phase 1: [2][TPS][P][QA][1 KiB]
  auto bgrp = [](int col, int g) { return col * 64 + 16 * (g ^ ((col >> 1) & 3)); };
  unsigned char* Hs = smem_ru;                 // phase 2: [P][nck1][BN][64 B] (aliases Bs and As)

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int nt_idx = wg % a.ntn;
  const int b = wg / a.ntn;
  const int n0 = nt_idx * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM;
  const int wn = wave / WM;

  const unsigned long long xb_u = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned xb_lo = __builtin_amdgcn_readfirstlane((unsigned)xb_u);
  const unsigned xb_hi = __builtin_amdgcn_readfirstlane((unsigned)(xb_u >> 32));
  const int xbytes = __builtin_amdgcn_readfirstlane(a.Cin * a.Tin * 4);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long long)xb_hi << 32) | xb_lo), 0, xbytes, 0x00020000);
  const int in0 = n0 - a.pl;

  const int K = a.K;
  const int kst = (K + TPS - 1) / TPS;  // phase-1 K-steps per chunk
  const int nsteps = a.nchunks * kst;
  const int a_pieces = P * QA;

  auto issue_a = [&](const float* w, int step, int buf) {
    const int c = step / kst, t0 = (step - c * kst) * TPS;
    const int n = (K - t0 < TPS ? K - t0 : TPS) * a_pieces;
    const unsigned char* src = reinterpret_cast<const unsigned char*>(w) + (long long)(c * K + t0) * (a_pieces * 1024);
    unsigned char* dst = As + buf * (TPS * a_pieces * 1024);
    if (!BC_DOK(c < a.nchunks && t0 * a_pieces + n <= K * a_pieces)) return;  // debug build: inside the packed k7 weights
    for (int q = wave; q < n; q += NW)
      __builtin_amdgcn_global_load_lds((const void*)(src + q * 1024 + lane * 16), (lds_void_t)(dst + q * 1024),
                                       16, 0, 0);
  };

  const int bp = (tid >> 5) & 15;
  const int bcl = tid & 31;
  const int bcg = tid >> 9;  // 0 with 8 waves
  auto bcol = [&](int i) { return bcl + 32 * (i * NCG + bcg); };
  float bv0[CI], bv1[CI];
  auto load_b = [&](int chunk) {
    const int ci0 = chunk * X6_BKC + 2 * bp;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcol(i);
      const int ti = in0 + col;
      const bool tin = col < ncol && ti >= 0 && ti < a.Tin;
      const unsigned o0 = (tin && ci0 < a.Cin) ? (unsigned)((ci0 * a.Tin + ti) * 4) : 0xfffffff0u;
      const unsigned o1 = (tin && ci0 + 1 < a.Cin) ? (unsigned)(((ci0 + 1) * a.Tin + ti) * 4) : 0xfffffff0u;
      bv0[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o0, 0, 0));
      bv1[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o1, 0, 0));
    }
  };
  auto bmax_publish = [&](int par) {
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const unsigned u0 = __float_as_uint(fabsf(bv0[i])), u1 = __float_as_uint(fabsf(bv1[i]));
      m = m > u0 ? m : u0;
      m = m > u1 ? m : u1;
    }
    m = wave_max_u32(m);
    if (lane == 0) smax[par][wave] = m;
  };
  auto bmax_scale = [&](int par) {
    unsigned m = smax[par][0];
#pragma unroll
    for (int w = 1; w < NW; ++w) m = m > smax[par][w] ? m : smax[par][w];
    return h3_scale_from_bits(__builtin_amdgcn_readfirstlane(m));
  };
  float xs = 1.f;  // P == 2: scale of the staged k=7 input chunk and of the phase-1 accumulator
  // snake on load (r.isa): activate the thread's two staged channels of `chunk` in registers (out-of-range
  // loads read 0 and snake(0) = 0: the zero padding of the activated signal, as the reference pads it)
  auto activate_b = [&](int chunk) {
    if (!r.isa || BC_ABL(r.dbg, 16)) return;
    const int ci0 = chunk * X6_BKC + 2 * bp;
    const float a0 = ci0 < a.Cin ? r.isa[ci0] : 0.f, b0 = ci0 < a.Cin ? r.isb[ci0] : 0.f;
    const float a1 = ci0 + 1 < a.Cin ? r.isa[ci0 + 1] : 0.f, b1 = ci0 + 1 < a.Cin ? r.isb[ci0 + 1] : 0.f;
#pragma unroll
    for (int i = 0; i < CI; ++i) {  // the two channels as one packed pair (bit-identical to snake() on each)
      const f32x2 v = snake_pk((f32x2){bv0[i], bv1[i]}, (f32x2){a0, a1}, (f32x2){b0, b1});
      bv0[i] = v.x;
      bv1[i] = v.y;
    }
  };
  auto store_b = [&]() {
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcol(i);
      if (col < ncol) {
        if constexpr (P == 2) {
          unsigned h, m;
          split2_h(bv0[i] * xs, bv1[i] * xs, h, m);
          unsigned char* p = Bs + bgrp(col, bp >> 2) + (bp & 3) * 4;
          *reinterpret_cast<unsigned*>(p) = h;
          *reinterpret_cast<unsigned*>(p + bplane) = m;
          continue;
        }
        if constexpr (P == 1) {
          *reinterpret_cast<unsigned*>(Bs + bgrp(col, bp >> 2) + (bp & 3) * 4) = pk_bf16(bv0[i], bv1[i]);
          continue;
        }
        unsigned h, m, l;
        split2(bv0[i], bv1[i], h, m, l);
        unsigned char* p = Bs + bgrp(col, bp >> 2) + (bp & 3) * 4;
        *reinterpret_cast<unsigned*>(p) = h;
        *reinterpret_cast<unsigned*>(p + bplane) = m;
        *reinterpret_cast<unsigned*>(p + 2 * bplane) = l;
      }
    }
  };

  // ---------------- phase 1: h = conv7(x_act), weights as the MFMA A operand ----------------
  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int col_lane = wn * NT * 16 + (lane & 15);

  // P == 2: next chunk's scale = min(current, its block scale); the accumulator follows exactly
  auto h3_next_scale = [&](int par) {
    const float sn = bmax_scale(par);
    if (sn < xs) {
      const float rr = sn / xs;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] *= rr;
      xs = sn;
    }
  };

  issue_a(a.w, 0, 0);
  load_b(0);
  activate_b(0);
  if constexpr (P == 2) {
    bmax_publish(0);
    lds_barrier();
    xs = bmax_scale(0);
  }
  store_b();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();


  // phase-2 wave geometry
  const bool p2 = wave < QA * NPW;
  const int mq = wave % QA, jg = wave / QA;

  for (int c = 0; c < a.nchunks; ++c) {
    for (int tp = 0; tp < kst; ++tp) {
      const int step = c * kst + tp;
      if (step + 1 < nsteps && !BC_ABL(r.dbg, 1)) issue_a(a.w, step + 1, (step + 1) & 1);
      if (tp == 0 && c + 1 < a.nchunks && !BC_ABL(r.dbg, 2)) {
        dma_issue_order();  // the next chunk's loads stay behind the copy (the counted wait below)
        load_b(c + 1);
      }
#pragma unroll
      for (int tt = 0; tt < TPS; ++tt) {
      const int tap = tp * TPS + tt;
      if (TPS > 1 && tap >= K) break;
      if (BC_ABL(r.dbg, 32)) break;
      const unsigned char* Ab = As + (step & 1) * (TPS * a_pieces * 1024) + tt * (a_pieces * 1024);
      const unsigned char* Bcol = Bs + bgrp(col_lane + tap * a.d, lane >> 4);
      frag_t bf[NT][P];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int p = 0; p < P; ++p)
          bf[j][p] = *reinterpret_cast<const frag_t*>(Bcol + j * 16 * 64 + p * bplane);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const unsigned char* Aq = Ab + (wm * MT + i) * 1024 + lane * 16;
        const frag_t a0 = *reinterpret_cast<const frag_t*>(Aq);
        if constexpr (P == 2) {
          const frag_t a1 = *reinterpret_cast<const frag_t*>(Aq + QA * 1024);
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            floatx4 t = acc[i][j];
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, bf[j][0], t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bf[j][1], t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, bf[j][0], t, 0, 0, 0);
            acc[i][j] = t;
          }
          continue;
        } else if constexpr (P == 1) {
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[j][0], acc[i][j], 0, 0, 0);
        } else {
        const bf16x8_t a1 = *reinterpret_cast<const bf16x8_t*>(Aq + QA * 1024);
        const bf16x8_t a2 = *reinterpret_cast<const bf16x8_t*>(Aq + 2 * QA * 1024);
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          floatx4 t = acc[i][j];
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bf[j][0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[j][1], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[j][2], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[j][0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[j][1], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[j][0], t, 0, 0, 0);
          acc[i][j] = t;
        }
        }
      }
      }
      if (tp == kst - 1 && c + 1 < a.nchunks) {
        activate_b(c + 1);
        if constexpr (P == 2) bmax_publish((c + 1) & 1);
        lds_barrier();
        if constexpr (P == 2) h3_next_scale((c + 1) & 1);
        store_b();
      }
      if (tp == 0 && kst > 1 && c + 1 < a.nchunks)
        wait_vmcnt<2 * CI>();
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
    }
  }

  // ---------------- bridge: snake2(h + b7) -> 3 bf16 planes in LDS ----------------
  // this wave's phase-2 k=1 weight fragments (packed [chunk][plane][m-tile][lane][8]), loaded into
  // registers here so they land while the bridge runs
  frag_t w1f[KC1][P];
#pragma unroll
  for (int kc = 0; kc < KC1; ++kc)
#pragma unroll
    for (int p = 0; p < P; ++p)
      w1f[kc][p] = (p2 && kc < r.nck1 && BC_DOK(mq < QA))
                       ? *reinterpret_cast<const frag_t*>(reinterpret_cast<const unsigned char*>(r.w1) +
                                                          ((kc * P + p) * QA + mq) * 1024 + lane * 16)
                       : frag_t{};
  // (Hs overwrites Bs and As: every wave has passed the last step's barrier, no copy is in flight)
  const int C = a.Cout;
  if (C < r.nck1 * X6_BKC) {  // zero the pad channels of the last chunk (never written below)
    const int g0 = (C % X6_BKC) / 8;
    for (int idx = tid; idx < P * BN * 4; idx += NTHR) {
      const int p = idx / (BN * 4), n = (idx / 4) % BN, g = idx % 4;
      if (g >= g0)
        *reinterpret_cast<floatx4*>(Hs + p * r.hplane + (r.nck1 - 1) * (BN * 64) + hs_off(n, g)) =
            floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
  float hs = 1.f;  // P == 2: scale of the h tile (block maximum over all its channels and columns)
  if constexpr (P == 2) {
    // h = snake2(acc * (1 / (x scale * w7 row scale)) + b7), its block maximum, then the split below
    const float xinv = 1.f / xs;
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int co = wm * MT * 16 + i * 16 + (lane >> 4) * 4;
      if (co >= C) continue;
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {  // channels co + 2 pr, co + 2 pr + 1 as packed pairs (bit-identical)
        const int c0 = co + 2 * pr;
        const f32x2 bias = a.bias ? (f32x2){a.bias[c0], a.bias[c0 + 1]} : (f32x2){0.f, 0.f};
        const f32x2 sc = {a.wsc[c0] * xinv, a.wsc[c0 + 1] * xinv};
        const f32x2 sa = {r.s2a[c0], r.s2a[c0 + 1]}, sb = {r.s2b[c0], r.s2b[c0 + 1]};
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const f32x2 pre = (f32x2){acc[i][j][2 * pr], acc[i][j][2 * pr + 1]} * sc + bias;
          const f32x2 v = BC_ABL(r.dbg, 64) ? pre : snake_pk(pre, sa, sb);
          acc[i][j][2 * pr] = v.x;
          acc[i][j][2 * pr + 1] = v.y;
          const unsigned u0 = __float_as_uint(fabsf(v.x)), u1 = __float_as_uint(fabsf(v.y));
          m = m > u0 ? m : u0;
          m = m > u1 ? m : u1;
        }
      }
    }
    m = wave_max_u32(m);
    if (lane == 0) smax[0][wave] = m;  // slot 0: its last phase-1 reader passed the final barrier
    lds_barrier();
    hs = bmax_scale(0);
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int co = wm * MT * 16 + i * 16 + (lane >> 4) * 4;  // 4 consecutive channels co..co+3
    if (co >= C) continue;
    if constexpr (P == 2) {
      unsigned char* hrow = Hs + (co / X6_BKC) * (BN * 64) + (co % 8) * 2;
      const int g = (co % X6_BKC) / 8;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = wn * NT * 16 + j * 16 + (lane & 15);
        unsigned h0, m0, h1, m1;
        split2_h(acc[i][j][0] * hs, acc[i][j][1] * hs, h0, m0);
        split2_h(acc[i][j][2] * hs, acc[i][j][3] * hs, h1, m1);
        unsigned char* dst = hrow + hs_off(n, g);
        *reinterpret_cast<u32x2_t*>(dst) = (u32x2_t){h0, h1};
        *reinterpret_cast<u32x2_t*>(dst + r.hplane) = (u32x2_t){m0, m1};
      }
      continue;
    }
    float bias[4], sa[4], sb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bias[q] = a.bias ? a.bias[co + q] : 0.f;
      sa[q] = r.s2a[co + q];
      sb[q] = r.s2b[co + q];
    }
    unsigned char* hrow = Hs + (co / X6_BKC) * (BN * 64) + (co % 8) * 2;
    const int g = (co % X6_BKC) / 8;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = wn * NT * 16 + j * 16 + (lane & 15);
      float v[4];
      const f32x2 lo = snake_pk((f32x2){acc[i][j][0] + bias[0], acc[i][j][1] + bias[1]}, (f32x2){sa[0], sa[1]},
                                (f32x2){sb[0], sb[1]});
      const f32x2 hi = snake_pk((f32x2){acc[i][j][2] + bias[2], acc[i][j][3] + bias[3]}, (f32x2){sa[2], sa[3]},
                                (f32x2){sb[2], sb[3]});
      v[0] = lo.x, v[1] = lo.y, v[2] = hi.x, v[3] = hi.y;
      if constexpr (P == 1) {
        *reinterpret_cast<u32x2_t*>(hrow + hs_off(n, g)) = (u32x2_t){pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3])};
        continue;
      }
      unsigned h0, m0, l0, h1, m1, l1;
      split2(v[0], v[1], h0, m0, l0);
      split2(v[2], v[3], h1, m1, l1);
      unsigned char* dst = hrow + hs_off(n, g);
      *reinterpret_cast<u32x2_t*>(dst) = (u32x2_t){h0, h1};
      *reinterpret_cast<u32x2_t*>(dst + r.hplane) = (u32x2_t){m0, m1};
      *reinterpret_cast<u32x2_t*>(dst + 2 * r.hplane) = (u32x2_t){l0, l1};
    }
  }
  // the epilogue's residual (the unit's skip input x_raw): the 16-byte groups of the tiles this wave finishes in
  // phase 2, issued once h is in LDS (the accumulators are dead: no spills) so they land under phase 2 (the epilogue
  // loaded them itself: one exposed HBM round trip per workgroup, 20 % of a C = 96 unit in the round-4 ablation,
  // profiles/r04e_ru_ablation.txt)
  floatx4 rpre[NTW];
  {
    const float* rb = e.res ? e.res + (long long)b * e.rbs : nullptr;
    const int co = mq * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int nb = n0 + (jg * NTW + j) * 16 + (lane >> 4) * 4;
      rpre[j] = floatx4{0.f, 0.f, 0.f, 0.f};
      if (p2 && rb && e.vec && co < e.Cout && nb + 3 < e.Nout &&
          BC_DOK((long long)co * e.yT + e.ooff + nb + 3 < e.rbs))
        rpre[j] = *reinterpret_cast<const floatx4*>(rb + (long long)co * e.yT + e.ooff + nb);
    }
  }
  lds_barrier();

  // ---------------- phase 2: y = conv1(h_act), input as the MFMA A operand ----------------
  // Wave (mq, jg) computes m-tile mq for n-tiles [jg * NTW, (jg + 1) * NTW) from its register-resident
  // k=1 weights; Hs is read-only here, so phase 2 runs without a barrier.
  if (p2 && !BC_ABL(r.dbg, 8)) {
    floatx4 acc2[1][NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc2[0][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int n = (jg * NTW + j) * 16 + (lane & 15);
#pragma unroll
      for (int kc = 0; kc < KC1; ++kc) {
        if (kc >= r.nck1) break;
        const unsigned char* src = Hs + kc * (BN * 64) + hs_off(n, lane >> 4);
        frag_t bf[P];
#pragma unroll
        for (int p = 0; p < P; ++p) bf[p] = *reinterpret_cast<const frag_t*>(src + p * r.hplane);
        floatx4 t = acc2[0][j];
        if constexpr (P == 2) {
          t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[0], w1f[kc][1], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[1], w1f[kc][0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[0], w1f[kc][0], t, 0, 0, 0);
          acc2[0][j] = t;
          continue;
        } else if constexpr (P == 1) {
          acc2[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[0], w1f[kc][0], t, 0, 0, 0);
        } else {
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[0], w1f[kc][2], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[1], w1f[kc][1], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[2], w1f[kc][0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[0], w1f[kc][1], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[1], w1f[kc][0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[0], w1f[kc][0], t, 0, 0, 0);
        acc2[0][j] = t;
        }
      }
    }
    if (BC_ABL(r.dbg, 4)) {
      if (acc2[0][0][0] == 1234.5f) e.y[0] = 0.f;  // keep the MFMAs alive
    } else {
      conv_epilogue_res<NTW, P == 2>(e, acc2, b, mq * 16, n0 + jg * NTW * 16, lane, 1.f / hs, rpre);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
// Candidate x6 tiles (cfg ids of conv1d_x6.hip) with one m-group covering C, in order of preference
// (96 x 128 first: the tile the standalone k=7 conv runs fastest at C = 96).  Only configurations
// with <= 80 KB of LDS (two workgroups per CU, NT = 1 so 128 VGPRs suffice) are used: measured on
// MI355X, the one-launch unit only beats the two separate convs when a second workgroup's MFMAs hide
// each workgroup's operand loads and epilogue stores (at one workgroup per CU it was a wash at C = 48
// and 96 and 8% slower at C = 192, profiles/r01_x6b_layer_profile.txt vs r01_resunit_v1_layers.txt).
// h3 / bf16 at C = 96 take 123 first (the same 96 x 128 tile as 2 x 4 waves of 48 x 32: 10 instead of 14 LDS
// fragment reads per K32 unit, bit-identical outputs): 4-6 % per unit (profiles/r03m_ru_tiles.txt); x6 is
// neutral there (7.05 vs 7.08 ms) and keeps 109.  The 48-row bf16 tiles with more columns per wave (106, 124)
// need more than 128 VGPRs (one workgroup per CU) and run 1.8-2.1x slower than 111.
// Measured and not kept (round 4, profiles/r04d_resunit_w16_rejected.txt): the same units on 16-wave tiles, one
// 1024-thread workgroup per CU (96 x 256 at C = 96: 5.76 -> 6.36 ms, 6.09 with four taps per K-step; 48 x 512 at
// C = 48: 6.15 ms against the strip kernel's 4.52, with 14-28 spilled VGPRs): the kernel takes 16-wave tiles, the
// table has none.
static const int kRUCandidates[] = {109, 111, 110, 116, 112, 113, 117, 106, 104, 105, 123, 124};
static const int kRUCandidatesP12[] = {123, 109, 111, 110, 116, 112, 113, 117, 106, 104, 105, 124};
constexpr size_t RU_LDS_MAX = 80 * 1024;
// LDS budget of a candidate: two workgroups per CU for the 8-wave tiles, the whole CU for 16-wave ones
static size_t ru_lds_budget(const X6Tile& t) { return t.WM * t.WN == 16 ? 160 * 1024 : RU_LDS_MAX; }
// BC_RU_CFG forces one candidate tile (timing experiments; it must fit the 160 KiB of a CU).
static int ru_forced_cfg() {
  static const int v = [] {
    const char* e = getenv("BC_RU_CFG");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static size_t ru_lds(const X6Tile& t, int C, int d, int P, int* bplane, int* hplane, int tps = 1) {
  const int ncol = x6_ncol(t, 7, 1, d);
  *bplane = (ncol * 64 + 15) / 16 * 16;  // swizzled 64-B pitch (x6_common.h x6_pitch)
  *hplane = (C + X6_BKC - 1) / X6_BKC * x6_BN(t) * 64;
  const size_t ph1 = P * (size_t)*bplane + 2 * tps * P * (size_t)t.WM * t.MT * 1024;  // Bs + As
  const size_t ph2 = P * (size_t)*hplane;                                               // Hs
  return ph1 > ph2 ? ph1 : ph2;
}

// k=7 taps per phase-1 K-step (h3), measured (profiles/r01g_ru_tps_prefetch_sweep.txt): 4 at C <= 64
// (C = 48: -4 %), else 2 (C = 96: -2 %; 4 is 1.5x slower there), each only where the A buffers keep
// the unit within the two-workgroups-per-CU LDS budget.  x6 (round 5): 2 at C <= 64 -- the C = 48 unit 6.07 / 6.07 /
// 6.14 -> 5.86 / 5.91 / 5.97 ms at d = 1 / 3 / 9 (profiles/r05i_ru48_tps2.txt); the same K order per output, so
// bit-identical; C = 96 keeps 1 (two taps exceed the 80 KiB budget).  BC_RU_TPS forces 1 / 2 / 4 (timing experiments).
static int ru_tps(const X6Tile& t, int C, int d, int P) {
  static const int forced = [] {
    const char* e = getenv("BC_RU_TPS");
    return e ? atoi(e) : 0;
  }();
  int bp, hp;
  if (P == 3) {  // x6: two taps per K-step on the C = 48 tile (MT 3, NT 1, WM 1) only: launch_ru has no other x6 TPS-2
                 // kernel, so any other tile's LDS size, launched template and kernel name are those of one tap
    const bool t48 = t.MT == 3 && t.NT == 1 && t.WM == 1;
    return t48 && C <= 64 && forced != 1 && forced != 4 && ru_lds(t, C, d, P, &bp, &hp, 2) <= ru_lds_budget(t) ? 2 : 1;
  }
  if (forced == 1 || forced == 2 || forced == 4) return forced;
  for (int tps : {4, 2})
    if ((tps < 4 || C <= 64) && ru_lds(t, C, d, P, &bp, &hp, tps) <= ru_lds_budget(t)) return tps;
  return 1;
}

// mode 1 (x6) -> cfg 1xx, mode 2 (bf16) -> cfg 2xx, mode 3 (h3) -> cfg 3xx (same tile table)
int resunit_select_cfg(int C, int d, int mode) {
  if (mode < 1 || mode > 3 || C < 16 || C % 16 || d <= 0) return -1;
  const int P = mode == 3 ? 2 : mode == 2 ? 1 : 3;
  const int forced = ru_forced_cfg();
  // C = 192 (x6, bf16): the 16-wave 192 x 256 tile, k=1 weights streamed into registers (resunit_w16.hip)
  if (!forced && resunit_w16_ok(C, d, P)) return P == 1 ? 222 : 122;
  for (int cfg : (P == 3 ? kRUCandidates : kRUCandidatesP12)) {
    const X6Tile& t = x6_tile(cfg);
    if (x6_BM(t) != C) continue;
    if (d > RU_MAX_DIL) return -1;
    int bp, hp;
    const size_t lds = ru_lds(t, C, d, P, &bp, &hp);
    if (forced ? (cfg != forced || lds > 160 * 1024) : lds > ru_lds_budget(t)) continue;
    return cfg + (P == 2 ? 200 : P == 1 ? 100 : 0);
  }
  return -1;
}

// cfg is a one-launch unit tile for (C, d) in its mode: the selected one, or another candidate whose 16 * MT * WM
// rows cover C and whose LDS fits a CU (A/B timing and the tile bit-identity tests pick tiles explicitly).
bool resunit_cfg_ok(int cfg, int C, int d) {
  const int mode = cfg / 100;
  if (mode < 1 || mode > 3 || C < 16 || C % 16 || d <= 0 || d > RU_MAX_DIL) return false;
  if (cfg == resunit_select_cfg(C, d, mode)) return true;
  const int base = cfg % 100 + 100;
  bool cand = false;
  for (int c : kRUCandidates) cand = cand || c == base;
  if (!cand) return false;
  const X6Tile& t = x6_tile(base);
  const int P = mode == 3 ? 2 : mode == 2 ? 1 : 3;
  int bp, hp;
  return x6_BM(t) == C && ru_lds(t, C, d, P, &bp, &hp, ru_tps(t, C, d, P)) <= 160 * 1024;
}

template <int MT, int NT, int WM, int WN, int P>
static int launch_ru(ConvArgs& a, ConvArgs& e, RUExtra& r, int B, hipStream_t st) {
  constexpr int BN = 16 * NT * WN, NTHR = 64 * WM * WN;
  const X6Tile t{MT, NT, WM, WN};
  int bplane, hplane;
  const int tps = ru_tps(t, a.Cout, a.d, P);
  const size_t lds = ru_lds(t, a.Cout, a.d, P, &bplane, &hplane, tps);
  if (lds > 160 * 1024) return BC_ERR_UNSUPPORTED;
  a.win = x6_ncol(t, 7, 1, a.d);
  a.bstage = bplane;
  a.nchunks = (a.Cin + X6_BKC - 1) / X6_BKC;
  a.ntm = 1;
  a.ntn = (a.Nout + BN - 1) / BN;
  r.hplane = hplane;
  r.nck1 = (a.Cout + X6_BKC - 1) / X6_BKC;
  const long long nwg = (long long)a.ntn * B;
  if (nwg <= 0) return BC_OK;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  if ((long long)a.Cin * a.Tin * 4 > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  a.nwg = (int)nwg;
  if (P == 2) {  // 1 / row scales after each packed weight's planes (conv1d_x6.hip x6_pack_weight)
    constexpr int QA = MT * WM;
    a.wsc = reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(a.w) +
                                           (long long)a.nchunks * 7 * P * QA * 1024);
    e.wsc = reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(r.w1) +
                                           (long long)r.nck1 * P * QA * 1024);
  }
  if (P != 3 && tps == 4)
    hipLaunchKernelGGL((resunit_x6_kernel<MT, NT, WM, WN, P, (P != 3 ? 4 : 1)>), dim3(a.nwg), dim3(NTHR), lds, st, a, e, r);
  else if (tps == 2 && (P != 3 || (MT == 3 && NT == 1 && WM == 1)))  // (x6: the C = 48 tile only)
    hipLaunchKernelGGL((resunit_x6_kernel<MT, NT, WM, WN, P, (P != 3 || (MT == 3 && NT == 1 && WM == 1) ? 2 : 1)>),
                       dim3(a.nwg), dim3(NTHR), lds, st, a, e, r);
  else
    hipLaunchKernelGGL((resunit_x6_kernel<MT, NT, WM, WN, P>), dim3(a.nwg), dim3(NTHR), lds, st, a, e, r);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

int resunit_kernel_name(int cfg, int C, int d, char* buf, int n) {
  const int mode = cfg / 100;  // 1 x6, 2 bf16, 3 h3
  if (mode < 1 || mode > 3 || !resunit_cfg_ok(cfg, C, d)) return -1;
  if (cfg == 122 || cfg == 222) {  // resunit_w16.hip; the encoder flow activates on load unless BIGCODEC_RU_SNAKE_IN=0
    const char* e = getenv("BIGCODEC_RU_SNAKE_IN");      // (blocks.py)
    return snprintf(buf, n, "resunit_w16_kernel<%d, %d, true>", cfg == 122 ? 3 : 1, e && atoi(e) == 0 ? 0 : 2);
  }
  if (mode == 3 && resunit_rr_ok(C, d)) return resunit_rr_kernel_name(C, d, buf, n);
  const X6Tile& t = x6_tile(cfg);
  const int P = mode == 3 ? 2 : mode == 2 ? 1 : 3;
  return snprintf(buf, n, "resunit_x6_kernel<%d, %d, %d, %d, %d, %d>", t.MT, t.NT, t.WM, t.WN, P,
                  ru_tps(t, C, d, P));
}

int resunit_launch(const float* x_raw, const float* x_act, const float* w7, const float* b7, const float* s2a,
                   const float* s2b, const float* w1, const float* b1, const float* osa, const float* osb,
                   float* y, float* y2, int B, int C, int T, int d, int pl, int cfg, hipStream_t st,
                   const float* isa, const float* isb) {
  if (cfg >= 300 && cfg < 400 && resunit_rr_ok(C, d)) {  // h3 at C = 48: the register-weight / strip kernels
    const int rc = resunit_rr_launch(x_raw, x_act, w7, b7, s2a, s2b, w1, b1, osa, osb, y, y2, B, C, T, d, pl, st,
                                     isa, isb);
    if (rc != BC_ERR_UNSUPPORTED) return rc;
  }
  ConvArgs a{};
  a.x = x_act; a.w = w7; a.bias = b7;
  a.xbs = (long long)C * T;
  a.Cin = C; a.Tin = T; a.Cout = C; a.Nout = T;
  a.K = 7; a.s = 1; a.d = d; a.pl = pl;
  ConvArgs e{};
  e.bias = b1; e.res = x_raw; e.osa = osa; e.osb = osb; e.y = y; e.y2 = y2;
  e.ybs = (long long)C * T; e.rbs = e.ybs;
  e.Cout = C; e.Nout = T; e.yT = T; e.ostride = 1; e.ooff = 0; e.epi = 0;
  e.vec = conv_epilogue_vec_ok(e);
  static const int dbg = [] {
    const char* v = getenv("BC_RU_DEBUG");
    return v ? atoi(v) : 0;
  }();
  RUExtra r{w1, s2a, s2b, 0, 0, dbg, isa, isb};
  if (isa) a.x = x_raw;  // snake on load
  if (cfg == 122 || cfg == 222) {
    const int P = cfg == 122 ? 3 : 1;
    if (!resunit_w16_ok(C, d, P)) return BC_ERR_UNSUPPORTED;
    a.isa = isa;
    a.isb = isb;
    return resunit_w16_launch(a, e, w1, s2a, s2b, B, P, st);
  }
#define BC_RU_CASES(ID, MT, NT, WM, WN)                           \
  case 100 + ID: return launch_ru<MT, NT, WM, WN, 3>(a, e, r, B, st); \
  case 200 + ID: return launch_ru<MT, NT, WM, WN, 1>(a, e, r, B, st); \
  case 300 + ID: return launch_ru<MT, NT, WM, WN, 2>(a, e, r, B, st);
  switch (cfg) {
    BC_RU_CASES(11, 3, 1, 1, 8)
    BC_RU_CASES(10, 4, 1, 1, 8)
    BC_RU_CASES(16, 3, 1, 2, 4)
    BC_RU_CASES(12, 2, 1, 1, 8)
    BC_RU_CASES(13, 1, 1, 1, 8)
    BC_RU_CASES(9, 6, 1, 1, 8)
    BC_RU_CASES(6, 3, 2, 1, 8)
    BC_RU_CASES(4, 6, 2, 1, 8)
    BC_RU_CASES(5, 4, 2, 1, 8)
    BC_RU_CASES(17, 4, 1, 2, 4)
    BC_RU_CASES(23, 3, 2, 2, 4)
    BC_RU_CASES(24, 3, 4, 1, 8)
  }
#undef BC_RU_CASES
  return BC_ERR_ARG;
}

}  // namespace bc

BC_DEBUG_EXPORT(resunit_x6)
