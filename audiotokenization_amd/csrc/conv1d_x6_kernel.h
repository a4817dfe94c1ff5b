// Conv1d kernel template (x6 / h3 / bf16 operand planes) for gfx950: included by the per-precision
// translation units conv1d_x6_p{1,2,3}.hip (compiled in parallel); host logic in conv1d_x6.hip.
//
// Conv1d with fp32-accurate "3 x bf16" MFMA (x6 mode) for gfx950.
//
// Same GEMM and epilogue as conv1d.hip (reference: vq/module.py:11-72 and its callers), but the
// products run on v_mfma_f32_16x16x32_bf16 (16x the fp32 MFMA rate) with every fp32 operand split
// EXACTLY into three bf16 terms, v = v0 + v1 + v2 (round-to-nearest splits; 8+8+8 significant bits
// hold all 24 of an fp32 mantissa).  a*b is accumulated as the six terms with i+j <= 2:
//   a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0
// Every bf16*bf16 product is exact in fp32 and the MFMA accumulates in fp32; the three dropped terms
// are below 2^-26 |ab|.  The result has fp32-level error (DESIGN.md §4 measures it against fp64
// next to native fp32 accumulation) at 6/16 of the fp32-MFMA cost.
//
// Workgroup: 512 threads = WM x WN waves, each MT x NT 16x16 tiles; BM = 16*MT*WM, BN = 16*NT*WN.
// K is walked per (32-channel chunk, tap) = one K32 step.
//   A (weights): split and packed on the host, [mgroup][chunk][tap][plane][m-tile][lane][8 bf16];
//                one step's block (3 planes x WM*MT KiB) is copied by LDS-DMA, double-buffered.
//   B (input)  : per chunk, rows of the tile (incl. stride/dilation halo) are read from HBM into
//                registers (buffer loads: out-of-range -> 0), split into 3 bf16 planes and written
//                channel-contiguous ([col][32 ch], 80-B pitch: conflict-free b128 reads at stride 1)
//                so one ds_read_b128 gives a lane its 8 k-values.  The next chunk's loads are issued
//                at tap 0 and land while the current chunk's taps compute.
#pragma once
#include <type_traits>

#include "bc_common.h"
#include "bc_internal.h"
#include "conv_epilogue.h"
#include "x6_common.h"

namespace bc {

struct X6NoMid {};  // compute() without a mid-step hook

// P = operand planes: 3 (x6, fp32-accurate), 2 ("h3": two fp16 planes, three products, fp32-class
// accuracy at half the x6 MFMA count, x6_common.h) or 1 (plain bf16 products: the "bf16" precision
// mode of BASELINE config 5, activations still stored fp32).
// h3 scaling: each staged 32-channel B chunk gets a power-of-two scale from its block maximum (a wave
// reduction + an LDS exchange folded into the barrier in front of the chunk's store); the scale only
// ever decreases within a workgroup, the accumulator is rescaled (exactly) when it does, and the
// epilogue multiplies by 1 / (x scale * per-row weight scale).
// PW: pointwise (K = 1, the input tile is exactly BN columns) with the two-chunk-deep B prefetch.
// TPS: taps per K-step of the multi-tap path (1, 2, or 4 for bf16 on the 16-wave tile): one A copy, one wait and one barrier cover
// TPS (chunk, tap) units, i.e. BK = 32 * TPS per barrier.
// DB (multi-tap path, kst >= 3 for P == 2, >= 2 otherwise): two B buffers; chunk c + 1 is staged into the
// idle one during chunk c's K-steps (maxima published at step 1, split and stored at step 2 for h3 /
// step 1 otherwise) instead of behind an extra barrier at the chunk's last step, so the staging VALU and
// LDS writes overlap the other waves' MFMAs.
// B4 (multi-tap launches of stride-1 convs without phase decomposition, Tin % 4 == 0, 16-B aligned rows): the
// input chunk is read with 16-byte loads, each thread one channel pair x IT4 column quads (4 loads per thread on
// the 16-wave tile instead of 12 single-float loads), staged into the same LDS image with the same block maxima:
// outputs bit-identical to the single-float staging.
template <int MT, int NT, int WM, int WN, int P, bool PW, int TPS = 1, bool DB = false, bool B4 = false>
// NT == 1 tiles fit 128 VGPRs without spills: two 512-thread workgroups per CU where LDS allows, so
// one workgroup's epilogue stores and operand loads overlap the other's MFMAs.  WM * WN = 16: one
// 1024-thread workgroup (four waves per SIMD, <= 128 VGPRs).
__global__ void __launch_bounds__(64 * WM * WN, (WM * WN == 16 ? 1 : (NT == 1 ? 4 : 2))) conv1d_x6_kernel(ConvArgs a) {
  constexpr int BM = 16 * MT * WM;
  constexpr int BN = 16 * NT * WN;
  constexpr int QA = WM * MT;  // m-tiles per workgroup (1 KiB per plane each)
  constexpr int NW = WM * WN;  // waves: 8 or 16
  static_assert(NW == 8 || NW == 16, "512- or 1024-thread workgroups");
  constexpr int NCG = NW / 8;  // B staging column groups (16 channel pairs x 32 column lanes each)
  constexpr int CI = ((PW ? BN / 32 : X6_MAXCOL_ITERS) + NCG - 1) / NCG;  // 32-column B passes per thread
  constexpr int NQI = 4 * NW;  // B4: column quads per iteration (NW / 2 quad blocks of 8, 2 pair blocks of 8)
  // B4 iterations: ncol + 3 <= 4 * NQI * IT4 (pointwise: the input tile is the BN aligned columns)
  constexpr int IT4 = PW ? (BN / 4 + NQI - 1) / NQI : ((32 * X6_MAXCOL_ITERS + 6) / 4 + NQI - 1) / NQI;
  constexpr int NBL = B4 ? 2 * IT4 : 2 * CI;  // B load instructions per thread and chunk (the counted waits)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_x6[];
  __shared__ unsigned smax[2][NW];  // P == 2: per-wave maxima of the staged B chunk, by chunk parity
  typedef typename FragType<P>::type frag_t;

  const int ncol = a.win;                // columns of the input tile
  const int bplane = a.bstage;           // bytes per B plane (multiple of 16)
  const int bpitch = a.bpitch;           // x6_common.h x6_pitch
  const bool bswz = bpitch == 64;
  // byte offset of 16-B channel group g (channels 8g..8g+7 of the chunk) of column col
  auto bgrp = [&](int col, int g) { return col * bpitch + 16 * (bswz ? (g ^ ((col >> 1) & 3)) : g); };
  unsigned char* Bs = smem_x6;                            // [DB ? 2 : 1][P][ncol][bpitch]
  unsigned char* As = smem_x6 + (DB ? 2 : 1) * P * bplane;  // [2][TPS][P][QA][1 KiB]
  const unsigned char* Br = Bs;                           // B buffer the K-steps read

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int mt_idx = wg % a.ntm;
  const int rest = wg / a.ntm;
  const int nt_idx = rest % a.ntn;
  const int b = rest / a.ntn;
  const int m0 = mt_idx * BM;
  const int n0 = nt_idx * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM;
  const int wn = wave / WM;
  // MI355X_MICROARCH.md "Static priority for the younger half": the second-dispatched half of the workgroup loses
  // every VALU / issue arbitration to its SIMD partners; one s_setprio for it, no per-segment flips (A/B switch)
  if (NW == 16 && a.prio && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);

  const unsigned long long xb_u = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned xb_lo = __builtin_amdgcn_readfirstlane((unsigned)xb_u);
  const unsigned xb_hi = __builtin_amdgcn_readfirstlane((unsigned)(xb_u >> 32));
  const int xbytes = __builtin_amdgcn_readfirstlane((a.ps ? a.cin0 : a.Cin) * a.Tin * 4);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long long)xb_hi << 32) | xb_lo), 0, xbytes, 0x00020000);
  const int in0 = n0 * a.s - a.pl;
  const int tstep = a.ps ? a.ps : 1;  // input samples per B-tile column

  const int K = a.K;
  const int kst = (K + TPS - 1) / TPS;  // K-steps per chunk
  const int nsteps = a.nchunks * kst;
  const int a_pieces = P * QA;
  const unsigned char* wblk = reinterpret_cast<const unsigned char*>(a.w) +
                              (long long)mt_idx * a.nchunks * K * (a_pieces * 1024);

  // A copy of K-step `step` = taps [TPS * tp, TPS * tp + TPS) of chunk c (consecutive packed blocks)
  auto issue_a = [&](int step, int buf) {
    const int c = step / kst, t0 = (step - c * kst) * TPS;
    const int n = (K - t0 < TPS ? K - t0 : TPS) * a_pieces;
    const unsigned char* src = wblk + (long long)(c * K + t0) * (a_pieces * 1024);
    unsigned char* dst = As + buf * (TPS * a_pieces * 1024);
    // debug build: the copy stays inside this m-group's packed weights
    if (!BC_DOK(mt_idx < a.ntm && c < a.nchunks && t0 * a_pieces + n <= K * a_pieces)) return;
    for (int q = wave; q < n; q += NW)
      __builtin_amdgcn_global_load_lds((const void*)(src + q * 1024 + lane * 16), (lds_void_t)(dst + q * 1024),
                                       16, 0, 0);
  };

  // B staging: thread -> (channel pair p, column lane cl, column group g); columns cl + 32 * (i * NCG + g)
  const int bp = (tid >> 5) & 15;
  const int bcl = tid & 31;
  const int bcg = tid >> 9;  // 0 with 8 waves
  auto bcol = [&](int i) { return bcl + 32 * (i * NCG + bcg); };
  float bv0[CI], bv1[CI];
  auto load_b = [&](int chunk, float (&v0)[CI], float (&v1)[CI]) {
    const int ci0 = chunk * X6_BKC + 2 * bp;
    // channel (row) -> input channel and the input time of column 0; phase mode: row ci' is phase
    // r = ci' % ps of channel ci' / ps, column m reads sample (n0 + m) * ps + r - pl
    int ch0 = ci0, ch1 = ci0 + 1, tb0 = in0, tb1 = in0;
    if (a.ps) {
      ch0 = ci0 / a.ps;
      ch1 = (ci0 + 1) / a.ps;
      tb0 = n0 * a.ps + (ci0 - ch0 * a.ps) - a.pl;
      tb1 = n0 * a.ps + (ci0 + 1 - ch1 * a.ps) - a.pl;
    }
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcol(i);
      const int t0 = tb0 + col * tstep, t1 = tb1 + col * tstep;
      const bool cin = col < ncol;
      const unsigned o0 = (cin && ci0 < a.Cin && t0 >= 0 && t0 < a.Tin) ? (unsigned)((ch0 * a.Tin + t0) * 4) : 0xfffffff0u;
      const unsigned o1 =
          (cin && ci0 + 1 < a.Cin && t1 >= 0 && t1 < a.Tin) ? (unsigned)((ch1 * a.Tin + t1) * 4) : 0xfffffff0u;
      v0[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o0, 0, 0));
      v1[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o1, 0, 0));
    }
  };
  // B4 geometry: channel pair p4 of the chunk, column quad q = it * NQI + qb4 = input times tq0 + 4q .. + 3 =
  // tile columns 4q - r4 .. 4q - r4 + 3 (r4 = in0 mod 4, uniform per launch)
  const int r4 = ((in0 % 4) + 4) % 4;
  const int tq0 = in0 - r4;
  const int nq4 = (ncol + r4 + 3) >> 2;
  const int p4 = 8 * (wave & 1) + (lane & 7);
  const int qb4 = 8 * (wave >> 1) + (lane >> 3);
  floatx4 bq0[B4 ? IT4 : 1], bq1[B4 ? IT4 : 1];
  auto load_b4 = [&](int chunk, floatx4 (&v0)[B4 ? IT4 : 1], floatx4 (&v1)[B4 ? IT4 : 1]) {
    const int c0 = chunk * X6_BKC + 2 * p4;
#pragma unroll
    for (int it = 0; it < IT4; ++it) {
      const int q = it * NQI + qb4;
      const int t = tq0 + 4 * q;
      const bool ok = q < nq4 && t >= 0 && t < a.Tin;  // Tin % 4 == 0: a quad is wholly inside or outside
      // out of range: 0x80000000 > num_records (< 2^31), and the 16 bytes do not wrap the 32-bit offset
      const unsigned o0 = (ok && c0 < a.Cin) ? (unsigned)((c0 * a.Tin + t) * 4) : 0x80000000u;
      const unsigned o1 = (ok && c0 + 1 < a.Cin) ? (unsigned)(((c0 + 1) * a.Tin + t) * 4) : 0x80000000u;
      v0[it] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o0, 0, 0));
      v1[it] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o1, 0, 0));
    }
  };
  auto bmax_publish4 = [&](const floatx4 (&w0)[B4 ? IT4 : 1], const floatx4 (&w1)[B4 ? IT4 : 1], int par) {
    unsigned m = 0;  // over the tile's columns only (a quad's other times are not part of the staged tile)
#pragma unroll
    for (int it = 0; it < IT4; ++it) {
      const int col0 = 4 * (it * NQI + qb4) - r4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool in = col0 + j >= 0 && col0 + j < ncol;
        const unsigned u0 = in ? __float_as_uint(fabsf(w0[it][j])) : 0u, u1 = in ? __float_as_uint(fabsf(w1[it][j])) : 0u;
        m = m > u0 ? m : u0;
        m = m > u1 ? m : u1;
      }
    }
    m = wave_max_u32(m);
    if (lane == 0) smax[par][wave] = m;
  };
  // P == 2: publish this wave's block maximum of a chunk's staged values / read the block's scale
  auto bmax_publish = [&](const float (&w0)[CI], const float (&w1)[CI], int par) {
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const unsigned u0 = __float_as_uint(fabsf(w0[i])), u1 = __float_as_uint(fabsf(w1[i]));
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
  float xs = 1.f;  // P == 2: scale of the staged chunk and of the accumulator
  // channel pair pp of column col: split and stored into the P planes
  auto put = [&](int col, int pp, float v0, float v1, unsigned char* Bt, float sc) {
    unsigned char* p = Bt + bgrp(col, pp >> 2) + (pp & 3) * 4;
    if constexpr (P == 2) {
      unsigned h, m;
      split2_h(v0 * sc, v1 * sc, h, m);
      *reinterpret_cast<unsigned*>(p) = h;
      *reinterpret_cast<unsigned*>(p + bplane) = m;
      return;
    }
    const unsigned h = pk_bf16(v0, v1);
    *reinterpret_cast<unsigned*>(p) = h;
    if (P == 3) {
      const float r0 = v0 - bf_lo(h), r1 = v1 - bf_hi(h);
      const unsigned m = pk_bf16(r0, r1);
      const float s0 = r0 - bf_lo(m), s1 = r1 - bf_hi(m);
      const unsigned l = pk_bf16(s0, s1);
      *reinterpret_cast<unsigned*>(p + bplane) = m;
      *reinterpret_cast<unsigned*>(p + 2 * bplane) = l;
    }
  };
  auto store_b = [&](const float (&w0)[CI], const float (&w1)[CI], unsigned char* Bt, float sc) {
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcol(i);
      if (col < ncol) put(col, bp, w0[i], w1[i], Bt, sc);
    }
  };
  auto store_b4 = [&](const floatx4 (&w0)[B4 ? IT4 : 1], const floatx4 (&w1)[B4 ? IT4 : 1], unsigned char* Bt, float sc) {
#pragma unroll
    for (int it = 0; it < IT4; ++it) {
      const int col0 = 4 * (it * NQI + qb4) - r4;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (col0 + j >= 0 && col0 + j < ncol) put(col0 + j, p4, w0[it][j], w1[it][j], Bt, sc);
    }
  };
  // the staging steps on whichever register set the variant uses
  auto stage_load = [&](int chunk) {
    if constexpr (B4) load_b4(chunk, bq0, bq1);
    else load_b(chunk, bv0, bv1);
  };
  auto stage_max = [&](int par) {
    if constexpr (B4) bmax_publish4(bq0, bq1, par);
    else bmax_publish(bv0, bv1, par);
  };
  auto stage_store = [&](unsigned char* Bt, float sc) {
    if constexpr (B4) store_b4(bq0, bq1, Bt, sc);
    else store_b(bv0, bv1, Bt, sc);
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // P == 2, at a chunk boundary (the previous chunk's B tile is no longer read): the next chunk's
  // scale = min(current, its block scale); the accumulator follows exactly (powers of two)
  auto rescale_to = [&](float sn) {
    if (sn < xs) {
      const float r = sn / xs;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] *= r;
      xs = sn;
    }
  };
  auto h3_next_scale = [&](int par) { rescale_to(bmax_scale(par)); };

  const int col_lane = (wn * NT * 16 + (lane & 15)) * a.s;

  // one K32 unit: this wave's MT x NT tiles += A(buffer buf, slot tt) * B(tap-shifted columns); mid() (unless
  // X6NoMid) runs after m-tile 0's MFMAs
  const X6NoMid nomid{};
  auto compute = [&](int buf, int tt, int tap, auto&& mid) {
      const unsigned char* Ab = As + buf * (TPS * a_pieces * 1024) + tt * (a_pieces * 1024);
      // (n-tile j adds 16 * s columns: the swizzle of a stride-1 tile repeats every 8 columns)
      const unsigned char* Bcol = Br + bgrp(col_lane + tap * a.d, lane >> 4);
      frag_t bf[NT][P];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int p = 0; p < P; ++p)
          bf[j][p] = *reinterpret_cast<const frag_t*>(Bcol + j * 16 * a.s * bpitch + p * bplane);
      // A fragments one m-tile ahead (two register sets): m-tile i + 1's reads issue after m-tile i's
      // first n-tile of MFMAs (pinned by sched barriers), so the lgkmcnt(0) the compiler places before
      // m-tile i + 1 (pending LDS-DMA makes it count to zero) finds them landed instead of draining
      // fresh reads before every m-tile
      // (multi-tap tiles with NT > 1 and at most 24 accumulator tiles: the extra register set spills
      // in the others)
      // (x6 on the 16-wave tile: its three planes leave no room for the second set, 41 spilled VGPRs with it)
      constexpr bool APF = !PW && NT > 1 && MT * NT <= 24 && !(P == 3 && WM * WN == 16);
      frag_t af[2][P];
      auto load_a = [&](int i, frag_t (&d)[P]) {
        const unsigned char* Aq = Ab + (wm * MT + i) * 1024 + lane * 16;
#pragma unroll
        for (int p = 0; p < P; ++p) d[p] = *reinterpret_cast<const frag_t*>(Aq + p * QA * 1024);
      };
      load_a(0, af[0]);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int sl = APF ? (i & 1) : 0;  // without the prefetch one register set, as before
        if (!APF && i > 0) load_a(i, af[0]);
        auto prefetch = [&](int j) {
          if (APF && j == 1 && i + 1 < MT) {
            __builtin_amdgcn_sched_barrier(0);
            load_a(i + 1, af[(i + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        if (APF) __builtin_amdgcn_sched_barrier(0);  // m-tile i's MFMAs stay after m-tile i - 1's
        const frag_t a0 = af[sl][0];
        if constexpr (P == 2) {
          const frag_t a1 = af[sl][1];
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            prefetch(j);
            floatx4 t = acc[i][j];
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][1], a0, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][0], a1, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][0], a0, t, 0, 0, 0);
            acc[i][j] = t;
          }
        } else if constexpr (P == 1) {
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            prefetch(j);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a0, acc[i][j], 0, 0, 0);
          }
        } else {
          const frag_t a1 = af[sl][1];
          const frag_t a2 = af[sl][P - 1];
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            // operands swapped (input as A): the tile comes out transposed, see conv_epilogue.h
            prefetch(j);
            floatx4 t = acc[i][j];
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a2, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a1, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][P - 1], a0, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a1, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a0, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a0, t, 0, 0, 0);
            acc[i][j] = t;
          }
        }
        if constexpr (!std::is_same<std::decay_t<decltype(mid)>, X6NoMid>::value) {
          if (i == 0) {
            __builtin_amdgcn_sched_barrier(0);
            mid();
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
  };

  // prologue: A(step 0), B(chunk 0)
  issue_a(0, 0);
  stage_load(0);
  if constexpr (P == 2) {
    stage_max(0);
    lds_barrier();
    xs = bmax_scale(0);
  }
  stage_store(Bs, xs);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  if constexpr (PW) {
    // Pointwise conv (K = 1): one step per chunk, so the B loads run two chunks ahead in two
    // register sets (chunk c + 2 is issued while chunk c computes and chunk c + 1 is stored).
    float bw0[CI], bw1[CI];
    floatx4 bx0[B4 ? IT4 : 1], bx1[B4 ? IT4 : 1];  // B4: the second register set
    // the staging steps on a register set of the variant (float[CI] pairs or, B4, floatx4[IT4] pairs)
    auto ld = [&](int chunk, auto& v0, auto& v1) {
      if constexpr (B4) load_b4(chunk, v0, v1);
      else load_b(chunk, v0, v1);
    };
    auto mx = [&](auto& v0, auto& v1, int par) {
      if constexpr (B4) bmax_publish4(v0, v1, par);
      else bmax_publish(v0, v1, par);
    };
    auto st = [&](auto& v0, auto& v1) {
      if constexpr (B4) store_b4(v0, v1, Bs, xs);
      else store_b(v0, v1, Bs, xs);
    };
    auto step1 = [&](int c, auto& n0v, auto& n1v, auto& p0v, auto& p1v) {
      // chunk c + 1's registers (loaded one step ago) are consumed HERE, before this step's A copy: the compiler
      // does not count LDS-DMA copies, so its wait for them at the store below (or for the reuse of the other set
      // by chunk c + 2's loads) drained vmcnt to zero -- the fresh copy and chunk c + 2's loads included, one
      // full L2 + HBM round trip exposed per chunk.  Waited for here, they have had a whole step to land.
#pragma unroll
      for (int i = 0; i < (B4 ? IT4 : CI); ++i) asm volatile("" ::"v"(n0v[i]), "v"(n1v[i]));
      // the next chunk's copy and chunk c + 2's loads go out after the first m-tile of MFMAs (as on the k7 path)
      auto mid = [&]() {
        if (c + 1 < a.nchunks && !BC_ABL(a.dbg, 1)) issue_a(c + 1, (c + 1) & 1);
        dma_issue_order();  // chunk c + 2's loads stay behind the copy (the counted wait below)
        if (c + 2 < a.nchunks && !BC_ABL(a.dbg, 2)) ld(c + 2, p0v, p1v);
      };
      compute(c & 1, 0, 0, mid);
      if (c + 1 < a.nchunks) {
        if constexpr (P == 2) mx(n0v, n1v, (c + 1) & 1);
        lds_barrier();  // every wave is done reading this chunk's B tile
        if constexpr (P == 2) h3_next_scale((c + 1) & 1);
        if (!BC_ABL(a.dbg, 4)) st(n0v, n1v);
      }
      // the A copy of step c + 1 (issued before the NBL loads of chunk c + 2) must have landed
      if (c + 2 < a.nchunks)
        wait_vmcnt<NBL>();
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
    };
    if constexpr (B4) {
      if (a.nchunks > 1) ld(1, bx0, bx1);
      for (int c = 0; c < a.nchunks; c += 2) {
        step1(c, bx0, bx1, bq0, bq1);
        if (c + 1 < a.nchunks) step1(c + 1, bq0, bq1, bx0, bx1);
      }
    } else {
      if (a.nchunks > 1) ld(1, bw0, bw1);
      for (int c = 0; c < a.nchunks; c += 2) {
        step1(c, bw0, bw1, bv0, bv1);
        if (c + 1 < a.nchunks) step1(c + 1, bv0, bv1, bw0, bw1);
      }
    }
  } else {
    const bool prio = BC_ABL(a.dbg, 16);
    constexpr int DB_STORE = P == 2 ? 2 : 1;  // DB: K-step of chunk c that stores chunk c + 1
    for (int c = 0; c < a.nchunks; ++c) {
      float xn = xs;  // DB: scale of chunk c + 1
      if constexpr (DB) Br = Bs + (c & 1) * P * bplane;
      for (int tp = 0; tp < kst; ++tp) {
        const int step = c * kst + tp;
        if constexpr (B4 && TPS == 1) {
          // the next step's copy and (step 0 of a chunk) the next chunk's loads, issued after this step's first
          // m-tile of MFMAs: every wave leaves the barrier at once, and issuing the copies first held each SIMD's
          // matrix pipe idle for their issue cost (one-tap B4 steps only: the single-float staging's registers
          // spilled when live across the MFMAs)
          auto mid = [&]() {
            if (step + 1 < nsteps && !BC_ABL(a.dbg, 1)) issue_a(step + 1, (step + 1) & 1);
            if (tp == 0 && c + 1 < a.nchunks && !BC_ABL(a.dbg, 2)) {
              dma_issue_order();  // the next chunk's loads stay behind the copy (the counted wait below)
              stage_load(c + 1);
            }
          };
          if (prio) __builtin_amdgcn_s_setprio(1);
          compute(step & 1, 0, tp, mid);
        } else {
          if (step + 1 < nsteps && !BC_ABL(a.dbg, 1)) issue_a(step + 1, (step + 1) & 1);
          if (tp == 0 && c + 1 < a.nchunks && !BC_ABL(a.dbg, 2)) {
            dma_issue_order();  // the next chunk's loads stay behind the copy (the counted wait below)
            stage_load(c + 1);
          }
          if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int tt = 0; tt < TPS; ++tt) {
            const int tap = tp * TPS + tt;
            if (TPS == 1 || tap < K) compute(step & 1, tt, tap, nomid);
          }
        }
        if (prio) __builtin_amdgcn_s_setprio(0);
        if constexpr (DB) {
          // the idle buffer was last read in chunk c - 1 (every wave passed chunk c's first barrier)
          if (c + 1 < a.nchunks) {
            if (P == 2 && tp == 1) stage_max((c + 1) & 1);  // read at step 2, after a barrier
            if (tp == DB_STORE) {
              if constexpr (P == 2) {
                const float sn = bmax_scale((c + 1) & 1);
                xn = sn < xs ? sn : xs;
              }
              if (!BC_ABL(a.dbg, 4)) stage_store(Bs + ((c + 1) & 1) * P * bplane, xn);
            }
          }
        } else if (tp == kst - 1 && c + 1 < a.nchunks) {
          if constexpr (P == 2) stage_max((c + 1) & 1);
          lds_barrier();  // every wave is done reading this chunk's B tile
          if constexpr (P == 2) h3_next_scale((c + 1) & 1);
          if (!BC_ABL(a.dbg, 4)) stage_store(Bs, xs);
        }
        // Only the next step's A copy (LDS-DMA, not tracked by the compiler) must have landed.  At
        // step 0 of a multi-step chunk the NBL B loads of the next chunk were issued after it and
        // may stay in flight (vmcnt retires in issue order); they are consumed at the chunk's last
        // step, where the compiler waits for their registers itself.
        if (tp == 0 && kst > 1 && c + 1 < a.nchunks)
          wait_vmcnt<NBL>();
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
      }
      if constexpr (DB && P == 2) rescale_to(xn);  // chunk c's products are all in acc
    }
  }

  if (!BC_ABL(a.dbg, 8)) {
    if constexpr (P == 2)  // (one m-tile per pass on the multi-tap paths: two spill there)
      conv_epilogue<MT, NT, true, PW ? 0 : 1>(a, acc, b, m0 + wm * MT * 16, n0 + wn * NT * 16, lane, 1.f / xs);
    else
      conv_epilogue<MT, NT>(a, acc, b, m0 + wm * MT * 16, n0 + wn * NT * 16, lane);
  }
}

// ------------------------------------------------------------------------------------------------
// conv1d_x6_body: the same main loop as a device function ending with the accumulators handed to `fin` (resunit_w16.hip's
// bridge into the k=1 conv of a one-launch ResidualUnit).  conv1d_x6_kernel keeps its own copy: built on this body (a
// lambda epilogue) the 256 x 256 x6 tile was register-allocated differently -- 816 B of scratch where the kernel above
// has none -- and that build faulted (memory aperture violation) on the phase-decomposed debug-model launch; the conv
// kernels' code stays the one measured in rounds 2-5.
// SWAP (default): the input fragment is the MFMA's A operand, so the tile comes out transposed (a lane holds four
// consecutive columns of one channel, conv_epilogue.h); !SWAP: weights as A, a lane holds four consecutive channels
// of one column (the layout resunit_w16's bridge writes to LDS).  Same six products in the same order either way.
// SIN: the input's Activation1d (Snake) applied to the staged chunk in registers before the split, so the producer
// writes the raw tensor alone; per-channel coefficients from a.isa / a.isb (SIN 1) or from LDS at byte a.sin_lds,
// [alpha_exp Cin][inv_beta Cin] (SIN 2, staged by the caller before the body's prologue barrier).
extern __shared__ __attribute__((aligned(16))) unsigned char smem_xb[];

template <int MT, int NT, int WM, int WN, int P, bool PW, int TPS, bool DB, bool B4, bool SWAP, int SIN, class Fin>
__device__ __forceinline__ void conv1d_x6_body(const ConvArgs& a, Fin&& fin) {
  static_assert(!SIN || (!PW && P != 2), "snake on load: x6 / bf16 multi-tap launches only (h3 scales the raw chunk)");
  constexpr int BM = 16 * MT * WM;
  constexpr int BN = 16 * NT * WN;
  constexpr int QA = WM * MT;  // m-tiles per workgroup (1 KiB per plane each)
  constexpr int NW = WM * WN;  // waves: 8 or 16
  static_assert(NW == 8 || NW == 16, "512- or 1024-thread workgroups");
  constexpr int NCG = NW / 8;  // B staging column groups (16 channel pairs x 32 column lanes each)
  constexpr int CI = ((PW ? BN / 32 : X6_MAXCOL_ITERS) + NCG - 1) / NCG;  // 32-column B passes per thread
  constexpr int NQI = 4 * NW;  // B4: column quads per iteration (NW / 2 quad blocks of 8, 2 pair blocks of 8)
  // B4 iterations: ncol + 3 <= 4 * NQI * IT4 (pointwise: the input tile is the BN aligned columns)
  constexpr int IT4 = PW ? (BN / 4 + NQI - 1) / NQI : ((32 * X6_MAXCOL_ITERS + 6) / 4 + NQI - 1) / NQI;
  constexpr int NBL = B4 ? 2 * IT4 : 2 * CI;  // B load instructions per thread and chunk (the counted waits)
  __shared__ unsigned smax[2][NW];  // P == 2: per-wave maxima of the staged B chunk, by chunk parity
  typedef typename FragType<P>::type frag_t;

  const int ncol = a.win;                // columns of the input tile
  const int bplane = a.bstage;           // bytes per B plane (multiple of 16)
  const int bpitch = a.bpitch;           // x6_common.h x6_pitch
  const bool bswz = bpitch == 64;
  // byte offset of 16-B channel group g (channels 8g..8g+7 of the chunk) of column col
  auto bgrp = [&](int col, int g) { return col * bpitch + 16 * (bswz ? (g ^ ((col >> 1) & 3)) : g); };
  unsigned char* Bs = smem_xb;                            // [DB ? 2 : 1][P][ncol][bpitch]
  unsigned char* As = smem_xb + (DB ? 2 : 1) * P * bplane;  // [2][TPS][P][QA][1 KiB]
  const unsigned char* Br = Bs;                           // B buffer the K-steps read

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int mt_idx = wg % a.ntm;
  const int rest = wg / a.ntm;
  const int nt_idx = rest % a.ntn;
  const int b = rest / a.ntn;
  const int m0 = mt_idx * BM;
  const int n0 = nt_idx * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM;
  const int wn = wave / WM;
  // MI355X_MICROARCH.md "Static priority for the younger half": the second-dispatched half of the workgroup loses
  // every VALU / issue arbitration to its SIMD partners; one s_setprio for it, no per-segment flips (A/B switch)
  if (NW == 16 && a.prio && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);

  const unsigned long long xb_u = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned xb_lo = __builtin_amdgcn_readfirstlane((unsigned)xb_u);
  const unsigned xb_hi = __builtin_amdgcn_readfirstlane((unsigned)(xb_u >> 32));
  const int xbytes = __builtin_amdgcn_readfirstlane((a.ps ? a.cin0 : a.Cin) * a.Tin * 4);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long long)xb_hi << 32) | xb_lo), 0, xbytes, 0x00020000);
  const int in0 = n0 * a.s - a.pl;
  const int tstep = a.ps ? a.ps : 1;  // input samples per B-tile column

  const int K = a.K;
  const int kst = (K + TPS - 1) / TPS;  // K-steps per chunk
  const int nsteps = a.nchunks * kst;
  const int a_pieces = P * QA;
  const unsigned char* wblk = reinterpret_cast<const unsigned char*>(a.w) +
                              (long long)mt_idx * a.nchunks * K * (a_pieces * 1024);

  // A copy of K-step `step` = taps [TPS * tp, TPS * tp + TPS) of chunk c (consecutive packed blocks)
  auto issue_a = [&](int step, int buf) {
    const int c = step / kst, t0 = (step - c * kst) * TPS;
    const int n = (K - t0 < TPS ? K - t0 : TPS) * a_pieces;
    const unsigned char* src = wblk + (long long)(c * K + t0) * (a_pieces * 1024);
    unsigned char* dst = As + buf * (TPS * a_pieces * 1024);
    // debug build: the copy stays inside this m-group's packed weights
    if (!BC_DOK(mt_idx < a.ntm && c < a.nchunks && t0 * a_pieces + n <= K * a_pieces)) return;
    for (int q = wave; q < n; q += NW)
      __builtin_amdgcn_global_load_lds((const void*)(src + q * 1024 + lane * 16), (lds_void_t)(dst + q * 1024),
                                       16, 0, 0);
  };

  // B staging: thread -> (channel pair p, column lane cl, column group g); columns cl + 32 * (i * NCG + g)
  const int bp = (tid >> 5) & 15;
  const int bcl = tid & 31;
  const int bcg = tid >> 9;  // 0 with 8 waves
  auto bcol = [&](int i) { return bcl + 32 * (i * NCG + bcg); };
  float bv0[CI], bv1[CI];
  auto load_b = [&](int chunk, float (&v0)[CI], float (&v1)[CI]) {
    const int ci0 = chunk * X6_BKC + 2 * bp;
    // channel (row) -> input channel and the input time of column 0; phase mode: row ci' is phase
    // r = ci' % ps of channel ci' / ps, column m reads sample (n0 + m) * ps + r - pl
    int ch0 = ci0, ch1 = ci0 + 1, tb0 = in0, tb1 = in0;
    if (a.ps) {
      ch0 = ci0 / a.ps;
      ch1 = (ci0 + 1) / a.ps;
      tb0 = n0 * a.ps + (ci0 - ch0 * a.ps) - a.pl;
      tb1 = n0 * a.ps + (ci0 + 1 - ch1 * a.ps) - a.pl;
    }
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcol(i);
      const int t0 = tb0 + col * tstep, t1 = tb1 + col * tstep;
      const bool cin = col < ncol;
      const unsigned o0 = (cin && ci0 < a.Cin && t0 >= 0 && t0 < a.Tin) ? (unsigned)((ch0 * a.Tin + t0) * 4) : 0xfffffff0u;
      const unsigned o1 =
          (cin && ci0 + 1 < a.Cin && t1 >= 0 && t1 < a.Tin) ? (unsigned)((ch1 * a.Tin + t1) * 4) : 0xfffffff0u;
      v0[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o0, 0, 0));
      v1[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o1, 0, 0));
    }
  };
  // B4 geometry: channel pair p4 of the chunk, column quad q = it * NQI + qb4 = input times tq0 + 4q .. + 3 =
  // tile columns 4q - r4 .. 4q - r4 + 3 (r4 = in0 mod 4, uniform per launch)
  const int r4 = ((in0 % 4) + 4) % 4;
  const int tq0 = in0 - r4;
  const int nq4 = (ncol + r4 + 3) >> 2;
  const int p4 = 8 * (wave & 1) + (lane & 7);
  const int qb4 = 8 * (wave >> 1) + (lane >> 3);
  floatx4 bq0[B4 ? IT4 : 1], bq1[B4 ? IT4 : 1];
  auto load_b4 = [&](int chunk, floatx4 (&v0)[B4 ? IT4 : 1], floatx4 (&v1)[B4 ? IT4 : 1]) {
    const int c0 = chunk * X6_BKC + 2 * p4;
#pragma unroll
    for (int it = 0; it < IT4; ++it) {
      const int q = it * NQI + qb4;
      const int t = tq0 + 4 * q;
      const bool ok = q < nq4 && t >= 0 && t < a.Tin;  // Tin % 4 == 0: a quad is wholly inside or outside
      // out of range: 0x80000000 > num_records (< 2^31), and the 16 bytes do not wrap the 32-bit offset
      const unsigned o0 = (ok && c0 < a.Cin) ? (unsigned)((c0 * a.Tin + t) * 4) : 0x80000000u;
      const unsigned o1 = (ok && c0 + 1 < a.Cin) ? (unsigned)(((c0 + 1) * a.Tin + t) * 4) : 0x80000000u;
      v0[it] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o0, 0, 0));
      v1[it] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o1, 0, 0));
    }
  };
  auto bmax_publish4 = [&](const floatx4 (&w0)[B4 ? IT4 : 1], const floatx4 (&w1)[B4 ? IT4 : 1], int par) {
    unsigned m = 0;  // over the tile's columns only (a quad's other times are not part of the staged tile)
#pragma unroll
    for (int it = 0; it < IT4; ++it) {
      const int col0 = 4 * (it * NQI + qb4) - r4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool in = col0 + j >= 0 && col0 + j < ncol;
        const unsigned u0 = in ? __float_as_uint(fabsf(w0[it][j])) : 0u, u1 = in ? __float_as_uint(fabsf(w1[it][j])) : 0u;
        m = m > u0 ? m : u0;
        m = m > u1 ? m : u1;
      }
    }
    m = wave_max_u32(m);
    if (lane == 0) smax[par][wave] = m;
  };
  // P == 2: publish this wave's block maximum of a chunk's staged values / read the block's scale
  auto bmax_publish = [&](const float (&w0)[CI], const float (&w1)[CI], int par) {
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const unsigned u0 = __float_as_uint(fabsf(w0[i])), u1 = __float_as_uint(fabsf(w1[i]));
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
  float xs = 1.f;  // P == 2: scale of the staged chunk and of the accumulator
  // channel pair pp of column col: split and stored into the P planes
  auto put = [&](int col, int pp, float v0, float v1, unsigned char* Bt, float sc) {
    unsigned char* p = Bt + bgrp(col, pp >> 2) + (pp & 3) * 4;
    if constexpr (P == 2) {
      unsigned h, m;
      split2_h(v0 * sc, v1 * sc, h, m);
      *reinterpret_cast<unsigned*>(p) = h;
      *reinterpret_cast<unsigned*>(p + bplane) = m;
      return;
    }
    const unsigned h = pk_bf16(v0, v1);
    *reinterpret_cast<unsigned*>(p) = h;
    if (P == 3) {
      const float r0 = v0 - bf_lo(h), r1 = v1 - bf_hi(h);
      const unsigned m = pk_bf16(r0, r1);
      const float s0 = r0 - bf_lo(m), s1 = r1 - bf_hi(m);
      const unsigned l = pk_bf16(s0, s1);
      *reinterpret_cast<unsigned*>(p + bplane) = m;
      *reinterpret_cast<unsigned*>(p + 2 * bplane) = l;
    }
  };

  // SIN: the staged chunk's two channels (c0, c0 + 1 of this thread's pair) as one packed pair through the Snake
  // (bit-identical to the producer epilogue's snake_pk on each; out-of-range loads read 0 and snake(0) = 0: the zero
  // padding of the activated signal, as the reference pads it)
  f32x2 sin_a = {0.f, 0.f}, sin_b = {0.f, 0.f};
  auto sin_coefs = [&](int chunk) {
    if constexpr (SIN == 1) {
      const int c0 = chunk * X6_BKC + 2 * (B4 ? p4 : bp);
      sin_a = (f32x2){c0 < a.Cin ? a.isa[c0] : 0.f, c0 + 1 < a.Cin ? a.isa[c0 + 1] : 0.f};
      sin_b = (f32x2){c0 < a.Cin ? a.isb[c0] : 0.f, c0 + 1 < a.Cin ? a.isb[c0 + 1] : 0.f};
    } else if constexpr (SIN == 2) {  // (Cin % 32 == 0: every pair is inside the table)
      const int c0 = chunk * X6_BKC + 2 * (B4 ? p4 : bp);
      const float* t = reinterpret_cast<const float*>(smem_xb + a.sin_lds);
      sin_a = *reinterpret_cast<const f32x2*>(t + c0);
      sin_b = *reinterpret_cast<const f32x2*>(t + a.Cin + c0);
    }
  };
  auto store_b = [&](const float (&w0)[CI], const float (&w1)[CI], unsigned char* Bt, float sc) {
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcol(i);
      if (col < ncol) {
        if constexpr (SIN) {
          const f32x2 v = BC_ABL(a.dbg, 32) ? (f32x2){w0[i], w1[i]} : snake_pk((f32x2){w0[i], w1[i]}, sin_a, sin_b);
          put(col, bp, v.x, v.y, Bt, sc);
        } else {
          put(col, bp, w0[i], w1[i], Bt, sc);
        }
      }
    }
  };
  auto store_b4 = [&](const floatx4 (&w0)[B4 ? IT4 : 1], const floatx4 (&w1)[B4 ? IT4 : 1], unsigned char* Bt, float sc) {
#pragma unroll
    for (int it = 0; it < IT4; ++it) {
      const int col0 = 4 * (it * NQI + qb4) - r4;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (col0 + j >= 0 && col0 + j < ncol) {
          if constexpr (SIN) {
            const f32x2 v = BC_ABL(a.dbg, 32) ? (f32x2){w0[it][j], w1[it][j]}
                                              : snake_pk((f32x2){w0[it][j], w1[it][j]}, sin_a, sin_b);
            put(col0 + j, p4, v.x, v.y, Bt, sc);
          } else {
            put(col0 + j, p4, w0[it][j], w1[it][j], Bt, sc);
          }
        }
    }
  };
  // the staging steps on whichever register set the variant uses
  auto stage_load = [&](int chunk) {
    if constexpr (B4) load_b4(chunk, bq0, bq1);
    else load_b(chunk, bv0, bv1);
  };
  auto stage_max = [&](int par) {
    if constexpr (B4) bmax_publish4(bq0, bq1, par);
    else bmax_publish(bv0, bv1, par);
  };
  auto stage_store = [&](unsigned char* Bt, float sc, int chunk) {
    if constexpr (SIN) sin_coefs(chunk);
    if constexpr (B4) store_b4(bq0, bq1, Bt, sc);
    else store_b(bv0, bv1, Bt, sc);
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // P == 2, at a chunk boundary (the previous chunk's B tile is no longer read): the next chunk's
  // scale = min(current, its block scale); the accumulator follows exactly (powers of two)
  auto rescale_to = [&](float sn) {
    if (sn < xs) {
      const float r = sn / xs;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] *= r;
      xs = sn;
    }
  };
  auto h3_next_scale = [&](int par) { rescale_to(bmax_scale(par)); };

  const int col_lane = (wn * NT * 16 + (lane & 15)) * a.s;

  // one K32 unit: this wave's MT x NT tiles += A(buffer buf, slot tt) * B(tap-shifted columns); mid() (unless
  // X6NoMid) runs after m-tile 0's MFMAs
  const X6NoMid nomid{};
  auto compute = [&](int buf, int tt, int tap, auto&& mid) {
      const unsigned char* Ab = As + buf * (TPS * a_pieces * 1024) + tt * (a_pieces * 1024);
      // (n-tile j adds 16 * s columns: the swizzle of a stride-1 tile repeats every 8 columns)
      const unsigned char* Bcol = Br + bgrp(col_lane + tap * a.d, lane >> 4);
      frag_t bf[NT][P];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int p = 0; p < P; ++p)
          bf[j][p] = *reinterpret_cast<const frag_t*>(Bcol + j * 16 * a.s * bpitch + p * bplane);
      // A fragments one m-tile ahead (two register sets): m-tile i + 1's reads issue after m-tile i's
      // first n-tile of MFMAs (pinned by sched barriers), so the lgkmcnt(0) the compiler places before
      // m-tile i + 1 (pending LDS-DMA makes it count to zero) finds them landed instead of draining
      // fresh reads before every m-tile
      // (multi-tap tiles with NT > 1 and at most 24 accumulator tiles: the extra register set spills
      // in the others)
      // (x6 on the 16-wave tile: its three planes leave no room for the second set, 41 spilled VGPRs with it)
      constexpr bool APF = !PW && NT > 1 && MT * NT <= 24 && !(P == 3 && WM * WN == 16);
      frag_t af[2][P];
      auto load_a = [&](int i, frag_t (&d)[P]) {
        const unsigned char* Aq = Ab + (wm * MT + i) * 1024 + lane * 16;
#pragma unroll
        for (int p = 0; p < P; ++p) d[p] = *reinterpret_cast<const frag_t*>(Aq + p * QA * 1024);
      };
      load_a(0, af[0]);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int sl = APF ? (i & 1) : 0;  // without the prefetch one register set, as before
        if (!APF && i > 0) load_a(i, af[0]);
        auto prefetch = [&](int j) {
          if (APF && j == 1 && i + 1 < MT) {
            __builtin_amdgcn_sched_barrier(0);
            load_a(i + 1, af[(i + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        if (APF) __builtin_amdgcn_sched_barrier(0);  // m-tile i's MFMAs stay after m-tile i - 1's
        const frag_t a0 = af[sl][0];
        if constexpr (P == 2) {
          const frag_t a1 = af[sl][1];
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            prefetch(j);
            floatx4 t = acc[i][j];
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][1], a0, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][0], a1, t, 0, 0, 0);
            t = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j][0], a0, t, 0, 0, 0);
            acc[i][j] = t;
          }
        } else if constexpr (P == 1) {
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            prefetch(j);
            acc[i][j] = SWAP ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a0, acc[i][j], 0, 0, 0)
                             : __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[j][0], acc[i][j], 0, 0, 0);
          }
        } else {
          const frag_t a1 = af[sl][1];
          const frag_t a2 = af[sl][P - 1];
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            // operands swapped (input as A): the tile comes out transposed, see conv_epilogue.h
            prefetch(j);
            floatx4 t = acc[i][j];
            if constexpr (SWAP) {
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a2, t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a1, t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][P - 1], a0, t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a1, t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][1], a0, t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][0], a0, t, 0, 0, 0);
            } else {
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bf[j][0], t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[j][1], t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[j][P - 1], t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bf[j][0], t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[j][1], t, 0, 0, 0);
              t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bf[j][0], t, 0, 0, 0);
            }
            acc[i][j] = t;
          }
        }
        if constexpr (!std::is_same<std::decay_t<decltype(mid)>, X6NoMid>::value) {
          if (i == 0) {
            __builtin_amdgcn_sched_barrier(0);
            mid();
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
  };

  // prologue: A(step 0), B(chunk 0)
  issue_a(0, 0);
  stage_load(0);
  if constexpr (P == 2) {
    stage_max(0);
    lds_barrier();
    xs = bmax_scale(0);
  }
  stage_store(Bs, xs, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  if constexpr (PW) {
    // Pointwise conv (K = 1): one step per chunk, so the B loads run two chunks ahead in two
    // register sets (chunk c + 2 is issued while chunk c computes and chunk c + 1 is stored).
    float bw0[CI], bw1[CI];
    floatx4 bx0[B4 ? IT4 : 1], bx1[B4 ? IT4 : 1];  // B4: the second register set
    // the staging steps on a register set of the variant (float[CI] pairs or, B4, floatx4[IT4] pairs)
    auto ld = [&](int chunk, auto& v0, auto& v1) {
      if constexpr (B4) load_b4(chunk, v0, v1);
      else load_b(chunk, v0, v1);
    };
    auto mx = [&](auto& v0, auto& v1, int par) {
      if constexpr (B4) bmax_publish4(v0, v1, par);
      else bmax_publish(v0, v1, par);
    };
    auto st = [&](auto& v0, auto& v1) {
      if constexpr (B4) store_b4(v0, v1, Bs, xs);
      else store_b(v0, v1, Bs, xs);
    };
    auto step1 = [&](int c, auto& n0v, auto& n1v, auto& p0v, auto& p1v) {
      // chunk c + 1's registers (loaded one step ago) are consumed HERE, before this step's A copy: the compiler
      // does not count LDS-DMA copies, so its wait for them at the store below (or for the reuse of the other set
      // by chunk c + 2's loads) drained vmcnt to zero -- the fresh copy and chunk c + 2's loads included, one
      // full L2 + HBM round trip exposed per chunk.  Waited for here, they have had a whole step to land.
#pragma unroll
      for (int i = 0; i < (B4 ? IT4 : CI); ++i) asm volatile("" ::"v"(n0v[i]), "v"(n1v[i]));
      // the next chunk's copy and chunk c + 2's loads go out after the first m-tile of MFMAs (as on the k7 path)
      auto mid = [&]() {
        if (c + 1 < a.nchunks && !BC_ABL(a.dbg, 1)) issue_a(c + 1, (c + 1) & 1);
        dma_issue_order();  // chunk c + 2's loads stay behind the copy (the counted wait below)
        if (c + 2 < a.nchunks && !BC_ABL(a.dbg, 2)) ld(c + 2, p0v, p1v);
      };
      compute(c & 1, 0, 0, mid);
      if (c + 1 < a.nchunks) {
        if constexpr (P == 2) mx(n0v, n1v, (c + 1) & 1);
        lds_barrier();  // every wave is done reading this chunk's B tile
        if constexpr (P == 2) h3_next_scale((c + 1) & 1);
        if (!BC_ABL(a.dbg, 4)) st(n0v, n1v);
      }
      // the A copy of step c + 1 (issued before the NBL loads of chunk c + 2) must have landed
      if (c + 2 < a.nchunks)
        wait_vmcnt<NBL>();
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
    };
    if constexpr (B4) {
      if (a.nchunks > 1) ld(1, bx0, bx1);
      for (int c = 0; c < a.nchunks; c += 2) {
        step1(c, bx0, bx1, bq0, bq1);
        if (c + 1 < a.nchunks) step1(c + 1, bq0, bq1, bx0, bx1);
      }
    } else {
      if (a.nchunks > 1) ld(1, bw0, bw1);
      for (int c = 0; c < a.nchunks; c += 2) {
        step1(c, bw0, bw1, bv0, bv1);
        if (c + 1 < a.nchunks) step1(c + 1, bv0, bv1, bw0, bw1);
      }
    }
  } else {
    const bool prio = BC_ABL(a.dbg, 16);
    constexpr int DB_STORE = P == 2 ? 2 : 1;  // DB: K-step of chunk c that stores chunk c + 1
    for (int c = 0; c < a.nchunks; ++c) {
      float xn = xs;  // DB: scale of chunk c + 1
      if constexpr (DB) Br = Bs + (c & 1) * P * bplane;
      for (int tp = 0; tp < kst; ++tp) {
        const int step = c * kst + tp;
        if constexpr (B4 && TPS == 1) {
          // the next step's copy and (step 0 of a chunk) the next chunk's loads, issued after this step's first
          // m-tile of MFMAs: every wave leaves the barrier at once, and issuing the copies first held each SIMD's
          // matrix pipe idle for their issue cost (one-tap B4 steps only: the single-float staging's registers
          // spilled when live across the MFMAs)
          auto mid = [&]() {
            if (step + 1 < nsteps && !BC_ABL(a.dbg, 1)) issue_a(step + 1, (step + 1) & 1);
            if (tp == 0 && c + 1 < a.nchunks && !BC_ABL(a.dbg, 2)) {
              dma_issue_order();  // the next chunk's loads stay behind the copy (the counted wait below)
              stage_load(c + 1);
            }
          };
          if (prio) __builtin_amdgcn_s_setprio(1);
          compute(step & 1, 0, tp, mid);
        } else {
          if (step + 1 < nsteps && !BC_ABL(a.dbg, 1)) issue_a(step + 1, (step + 1) & 1);
          if (tp == 0 && c + 1 < a.nchunks && !BC_ABL(a.dbg, 2)) {
            dma_issue_order();  // the next chunk's loads stay behind the copy (the counted wait below)
            stage_load(c + 1);
          }
          if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int tt = 0; tt < TPS; ++tt) {
            const int tap = tp * TPS + tt;
            if (TPS == 1 || tap < K) compute(step & 1, tt, tap, nomid);
          }
        }
        if (prio) __builtin_amdgcn_s_setprio(0);
        if constexpr (DB) {
          // the idle buffer was last read in chunk c - 1 (every wave passed chunk c's first barrier)
          if (c + 1 < a.nchunks) {
            if (P == 2 && tp == 1) stage_max((c + 1) & 1);  // read at step 2, after a barrier
            if (tp == DB_STORE) {
              if constexpr (P == 2) {
                const float sn = bmax_scale((c + 1) & 1);
                xn = sn < xs ? sn : xs;
              }
              if (!BC_ABL(a.dbg, 4)) stage_store(Bs + ((c + 1) & 1) * P * bplane, xn, c + 1);
            }
          }
        } else if (tp == kst - 1 && c + 1 < a.nchunks) {
          if constexpr (P == 2) stage_max((c + 1) & 1);
          lds_barrier();  // every wave is done reading this chunk's B tile
          if constexpr (P == 2) h3_next_scale((c + 1) & 1);
          if (!BC_ABL(a.dbg, 4)) stage_store(Bs, xs, c + 1);
        }
        // Only the next step's A copy (LDS-DMA, not tracked by the compiler) must have landed.  At
        // step 0 of a multi-step chunk the NBL B loads of the next chunk were issued after it and
        // may stay in flight (vmcnt retires in issue order); they are consumed at the chunk's last
        // step, where the compiler waits for their registers itself.
        if (tp == 0 && kst > 1 && c + 1 < a.nchunks)
          wait_vmcnt<NBL>();
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
      }
      if constexpr (DB && P == 2) rescale_to(xn);  // chunk c's products are all in acc
    }
  }

  fin(acc, b, m0, n0, wm, wn, lane, xs);
}

// ------------------------------------------------------------------------------------------------
// tile table and launch (shared with the host logic in conv1d_x6.hip)
// ------------------------------------------------------------------------------------------------
// cfg ids 100..: index into this table
inline constexpr X6Tile kX6Tiles[] = {
    {4, 4, 2, 4},  // 100: BM=128 BN=256  (Cout >= 128, stride 1)
    {4, 2, 2, 4},  // 101: BM=128 BN=128  (Cout >= 128, stride 2)
    {4, 2, 4, 2},  // 102: BM=256 BN=64   (Cout >= 256, stride >= 3)
    {2, 2, 4, 2},  // 103: BM=128 BN=64   (Cout >= 128, stride >= 3)
    {6, 2, 1, 8},  // 104: BM=96  BN=256
    {4, 2, 1, 8},  // 105: BM=64  BN=256
    {3, 2, 1, 8},  // 106: BM=48  BN=256
    {2, 2, 1, 8},  // 107: BM=32  BN=256
    {1, 2, 1, 8},  // 108: BM=16  BN=256
    {6, 1, 1, 8},  // 109: BM=96  BN=128
    {4, 1, 1, 8},  // 110: BM=64  BN=128
    {3, 1, 1, 8},  // 111: BM=48  BN=128
    {2, 1, 1, 8},  // 112: BM=32  BN=128
    {1, 1, 1, 8},  // 113: BM=16  BN=128
    {6, 2, 2, 4},  // 114: BM=192 BN=128  (Cout = 192k, stride <= 2)
    {6, 1, 2, 4},  // 115: BM=192 BN=64
    {3, 1, 2, 4},  // 116: BM=96  BN=64   (one-launch ResidualUnit at C = 96, two workgroups per CU)
    {4, 1, 2, 4},  // 117: BM=128 BN=64   (two workgroups per CU)
    {8, 2, 2, 4},  // 118: BM=256 BN=128  (h3: fits where the x6 planes did not)
    {4, 4, 4, 2},  // 119: BM=256 BN=128
    {6, 4, 2, 4},  // 120: BM=192 BN=256  (h3: 96 x 64 per wave)
    {8, 4, 2, 4},  // 121: BM=256 BN=256
    {6, 2, 2, 8},  // 122: BM=192 BN=256, 16 waves of 96 x 32 (h3 and bf16)
    // one-launch ResidualUnit only (resunit_x6.hip; the conv kernel does not instantiate them):
    {3, 2, 2, 4},  // 123: BM=96  BN=128, 48 x 32 per wave (C = 96: 10 instead of 14 LDS fragment reads per K32)
    {3, 4, 1, 8},  // 124: BM=48  BN=512, 48 x 64 per wave (bf16 C = 48: 7 reads per 12 MFMAs instead of 4 per 3)
};
constexpr int X6_NT = sizeof(kX6Tiles) / sizeof(kX6Tiles[0]);

inline size_t x6_lds(const X6Tile& t, int ncol, int planes, int s, int tps = 1, int bbufs = 1) {
  const size_t bplane = (size_t)((ncol * x6_pitch(s) + 15) / 16 * 16);
  return bbufs * planes * bplane + 2 * tps * planes * (size_t)t.WM * t.MT * 1024;
}

// h3 and bf16 kernels run the multi-tap path with two taps per K-step where the doubled A buffers fit the
// tile's LDS budget (measured: -4 % on the k7 convs, profiles/r01g_tps_sweep.txt); BC_X6_TPS=1 disables it.
inline int x6_tps() {
  static const int v = [] {
    const char* e = getenv("BC_X6_TPS");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  return v;
}

// BC_X6_PW=0 runs pointwise convs on the general kernel (A/B timing).
inline bool x6_pw_on() {
  static const bool v = [] {
    const char* e = getenv("BC_X6_PW");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// Which kernel variant a launch of tile t runs (shared by launch_x6 and bc_conv1d_kernel_name, so the
// name the roofline reports is the one that ran): the pointwise two-chunk-prefetch path (K = 1), two taps
// per K-step (h3 / bf16 multi-tap launches whose doubled A buffers fit), or one tap per K-step.
// BC_X6_DB=0 disables the double-buffered B tile (A/B timing).
inline bool x6_db_on() {
  static const bool v = [] {
    const char* e = getenv("BC_X6_DB");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// BC_X6_TPS4=0 keeps the bf16 16-wave tile at two taps per K-step (A/B timing).
inline bool x6_tps4_on() {
  static const bool v = [] {
    const char* e = getenv("BC_X6_TPS4");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// BC_X6_B4=0 keeps the single-float input staging everywhere (A/B timing).
inline bool x6_b4_on() {
  static const bool v = [] {
    const char* e = getenv("BC_X6_B4");
    return !e || atoi(e) != 0;
  }();
  return v;
}

struct X6Variant {
  bool pw;
  int tps;
  bool db;
  size_t lds;
  bool b4;  // 16-byte input staging (the launch also needs Tin % 4 == 0 and 16-B aligned rows, x6_b4_fits)
};
inline X6Variant x6_variant_base(const X6Tile& t, int P, int K, int s, int d) {
  const int ncol = x6_ncol(t, K, s, d);
  const size_t budget = t.NT > 1 ? 160 * 1024 : 80 * 1024;  // NT == 1: two workgroups per CU
  auto fits = [&](int tps, int bb) { return x6_lds(t, ncol, P, s, tps, bb) <= budget; };
  if (K == 1 && ncol == x6_BN(t) && x6_pw_on()) return {true, 1, false, x6_lds(t, ncol, P, s), false};
  const int min_kst = P == 2 ? 3 : 2;  // DB needs the store step after the maxima step
  // preference (profiles/r02_x6_db.txt): two taps per K-step over the double B buffer (fewer barriers
  // beat hidden staging: 192 x 256 k7 runs 2-3 % faster with TPS 2 than with DB at TPS 1); DB where only
  // one tap per step fits (256 x 256: k7 768 -4.5 %, k3 1536 -6 %); NT == 1 tiles never (slower, spills)
  const bool db = x6_db_on() && P <= 2 && t.NT > 1;
  const bool tps2 = P <= 2 && K > 1 && x6_tps() == 2;
  // bf16 on the 16-wave tile: one product per pair makes a two-tap K-step a third of h3's, too short to hide
  // the next step's A copy and the barrier; four taps per K-step over the double B buffer (k7: 2 K-steps per chunk)
  if (P == 1 && t.WM * t.WN == 16 && db && tps2 && x6_tps4_on() && (K + 3) / 4 >= min_kst && fits(4, 2))
    return {false, 4, true, x6_lds(t, ncol, P, s, 4, 2), false};
  if (db && tps2 && (K + 1) / 2 >= min_kst && fits(2, 2)) return {false, 2, true, x6_lds(t, ncol, P, s, 2, 2), false};
  if (tps2 && fits(2, 1)) return {false, 2, false, x6_lds(t, ncol, P, s, 2), false};
  if (db && K >= min_kst && fits(1, 2)) return {false, 1, true, x6_lds(t, ncol, P, s, 1, 2), false};
  return {false, 1, false, x6_lds(t, ncol, P, s), false};
}
// ps: the phase factor of a phase-decomposed strided conv (its rows gather s phases: no 16-byte staging)
inline X6Variant x6_variant(const X6Tile& t, int P, int K, int s, int d, int ps = 0) {
  X6Variant v = x6_variant_base(t, P, K, s, d);
  // 16-byte staging: the 16-wave tile's multi-tap launches, and the pointwise launches of the 16-wave tile and of
  // the 192 x 128 tile (whose 32-quad iteration covers its 128 columns)
  const bool pw_tile = t.WM * t.WN == 16 || (t.MT == 6 && t.NT == 2 && t.WM == 2 && t.WN == 4);
  v.b4 = s == 1 && ps == 0 && x6_b4_on() && (v.pw ? pw_tile : t.WM * t.WN == 16);
  return v;
}
// BC_X6_PRIO=1: static s_setprio(1) for the 16-wave tile's waves 8-15 (A/B timing)
inline int x6_prio() {
  static const int v = [] {
    const char* e = getenv("BC_X6_PRIO");
    return e ? atoi(e) : 0;
  }();
  return v;
}
inline bool x6_b4_fits(const ConvArgs& a) {
  return a.ps == 0 && a.s == 1 && a.Tin % 4 == 0 && a.xbs % 4 == 0 && ((unsigned long long)a.x & 15) == 0;
}

template <int MT, int NT, int WM, int WN, int P>
static int launch_x6(ConvArgs& a, int B, hipStream_t st) {
  constexpr int BM = 16 * MT * WM, BN = 16 * NT * WN, NTHR = 64 * WM * WN;
  const X6Tile t{MT, NT, WM, WN};
  const int ncol = x6_ncol(t, a.K, a.s, a.d);
  if (ncol > 32 * X6_MAXCOL_ITERS) return BC_ERR_UNSUPPORTED;
  a.ntm = (a.Cout + BM - 1) / BM;
  a.ntn = (a.Nout + BN - 1) / BN;
  a.nchunks = (a.Cin + X6_BKC - 1) / X6_BKC;
  a.win = ncol;
  a.bpitch = x6_pitch(a.s);
  a.bstage = (ncol * a.bpitch + 15) / 16 * 16;
  const long long nwg = (long long)a.ntm * a.ntn * B;
  if (nwg <= 0) return BC_OK;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  if ((long long)(a.ps ? a.cin0 : a.Cin) * a.Tin * 4 > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  a.nwg = (int)nwg;
  a.wsc = P == 2 ? reinterpret_cast<const float*>(reinterpret_cast<const unsigned char*>(a.w) +
                                                  (long long)a.ntm * a.nchunks * a.K * P * t.WM * t.MT * 1024)
                 : nullptr;
  const size_t lds = x6_lds(t, ncol, P, a.s);
  if (lds > 160 * 1024) return BC_ERR_UNSUPPORTED;
  const X6Variant v = x6_variant(t, P, a.K, a.s, a.d, a.ps);
  a.prio = x6_prio();
  constexpr int T2 = P <= 2 ? 2 : 1;
  constexpr bool D2 = P <= 2;
  if constexpr (WM * WN == 16) {  // 16-byte input staging: the 16-wave tile's multi-tap variant of each precision
    if (v.b4 && x6_b4_fits(a)) {
      constexpr int T4 = P == 1 ? 4 : P == 2 ? 2 : 1;
      constexpr bool D4 = P == 1;  // the k7 variants: bf16 4 taps over two B buffers, h3 2 taps, x6 1
      if (!v.pw && v.tps == T4 && v.db == D4) {  // (x6 pointwise launches also have tps 1, no DB: the PW path below)
        hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, false, T4, D4, true>), dim3(a.nwg), dim3(NTHR), v.lds,
                           st, a);
        BC_CHECK_LAUNCH();
        return BC_OK;
      }
    }
  }
  if constexpr (P == 1 && WM * WN == 16) {
    if (v.tps == 4) {
      hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, false, 4, true>), dim3(a.nwg), dim3(NTHR), v.lds, st, a);
      BC_CHECK_LAUNCH();
      return BC_OK;
    }
  }
  if constexpr (WM * WN == 16 || (MT == 6 && NT == 2 && WM == 2 && WN == 4)) {
    if (v.pw && v.b4 && x6_b4_fits(a)) {
      hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, true, 1, false, true>), dim3(a.nwg), dim3(NTHR), v.lds, st, a);
      BC_CHECK_LAUNCH();
      return BC_OK;
    }
  }
  if (v.pw)
    hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, true>), dim3(a.nwg), dim3(NTHR), v.lds, st, a);
  else if (v.db && v.tps == 2)
    hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, false, T2, D2>), dim3(a.nwg), dim3(NTHR), v.lds, st, a);
  else if (v.db)
    hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, false, 1, D2>), dim3(a.nwg), dim3(NTHR), v.lds, st, a);
  else if (v.tps == 2)
    hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, false, T2>), dim3(a.nwg), dim3(NTHR), v.lds, st, a);
  else
    hipLaunchKernelGGL((conv1d_x6_kernel<MT, NT, WM, WN, P, false>), dim3(a.nwg), dim3(NTHR), v.lds, st, a);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

// the 16-wave tile (every precision; x6 runs it without the A-fragment prefetch, which leaves 1 spilled VGPR
// at 128).  Measured and not kept (profiles/r02g_w16_tiles.txt, r02g_w16b.txt): 48 x 64 per wave (111 spilled
// VGPRs, 2.5x slower) and a 256 x 256 tile of 128 x 32 per wave (86-136 spilled VGPRs, 2.2-2.6x slower).
template <int P>
static int launch_x6_w16(ConvArgs& a, int B, hipStream_t st) {
  return launch_x6<6, 2, 2, 8, P>(a, B, st);
}

// launch tile index `tile` (kX6Tiles) with P operand planes; instantiated in conv1d_x6_p<P>.hip
template <int P>
int x6_launch_tile(ConvArgs& a, int B, int tile, hipStream_t st);

#define BC_X6_TILE_SWITCH(P)                                       \
  switch (tile) {                                                  \
    case 0: return launch_x6<4, 4, 2, 4, P>(a, B, st);             \
    case 1: return launch_x6<4, 2, 2, 4, P>(a, B, st);             \
    case 2: return launch_x6<4, 2, 4, 2, P>(a, B, st);             \
    case 3: return launch_x6<2, 2, 4, 2, P>(a, B, st);             \
    case 4: return launch_x6<6, 2, 1, 8, P>(a, B, st);             \
    case 5: return launch_x6<4, 2, 1, 8, P>(a, B, st);             \
    case 6: return launch_x6<3, 2, 1, 8, P>(a, B, st);             \
    case 7: return launch_x6<2, 2, 1, 8, P>(a, B, st);             \
    case 8: return launch_x6<1, 2, 1, 8, P>(a, B, st);             \
    case 9: return launch_x6<6, 1, 1, 8, P>(a, B, st);             \
    case 10: return launch_x6<4, 1, 1, 8, P>(a, B, st);            \
    case 11: return launch_x6<3, 1, 1, 8, P>(a, B, st);            \
    case 12: return launch_x6<2, 1, 1, 8, P>(a, B, st);            \
    case 13: return launch_x6<1, 1, 1, 8, P>(a, B, st);            \
    case 14: return launch_x6<6, 2, 2, 4, P>(a, B, st);            \
    case 15: return launch_x6<6, 1, 2, 4, P>(a, B, st);            \
    case 16: return launch_x6<3, 1, 2, 4, P>(a, B, st);            \
    case 17: return launch_x6<4, 1, 2, 4, P>(a, B, st);            \
    case 18: return launch_x6<8, 2, 2, 4, P>(a, B, st);            \
    case 19: return launch_x6<4, 4, 4, 2, P>(a, B, st);            \
    case 20: return launch_x6<6, 4, 2, 4, P>(a, B, st);            \
    case 21: return launch_x6<8, 4, 2, 4, P>(a, B, st);            \
    case 22: return launch_x6_w16<P>(a, B, st);                    \
    case 23:                                                       \
    case 24: return BC_ERR_UNSUPPORTED;                            \
  }                                                                \
  return BC_ERR_ARG;

}  // namespace bc
