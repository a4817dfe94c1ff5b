// x6 conv with REGISTER-resident weight fragments ("RA"): the multi-tap stride-1 convs (the ResidualUnit k7 convs,
// vq/module.py:59-65, 83) and the phase-decomposed strided ones (the EncoderBlock downsampling, vq/module.py:102-109)
// in the exact 3 x bf16 arithmetic of conv1d_x6_kernel.h, on a 192 x 256 tile of 8 waves (96 x 64 each).
//
// Why: the x6 operands are three planes, so in conv1d_x6_kernel<6, 2, 2, 8, 3> (16 waves, the A block of one K-step
// double-buffered in LDS: 2 x 36 KiB, plus the 50-60 KiB B tile) nothing else fits the 160 KiB LDS: one barrier per
// K-step (every 72 MFMAs of a wave), the next chunk's B tile staged behind an extra barrier with no MFMA beside it.
// Here each wave loads its own A fragments from L2 (global_load_dwordx4; the four waves of a row group read the same
// 18 KiB per K-step, mostly L1 hits) into 72 VGPRs that roll one K-step ahead: m-tile i's fragments of step s + 1 are
// requested right after their last use in step s.  The LDS holds only the B tile, double-buffered: chunk c + 1 is
// loaded into registers during chunk c - 1 (right after chunk c's planes were stored) and split + stored during
// chunk c's last K-step, and the ONLY barrier is at the end of a chunk (K = 7: one barrier per 7 x 144 MFMAs of a wave
// instead of per 72).
//
// Arithmetic: the same B planes (split2 of the same fp32 values), the same A planes (the cfg-120 / 122 packing: 12
// m-tiles of 16 rows per 192-row group, identical for both tiles), the same chunk-major, tap-minor K order and the
// same six-MFMA chain per output as conv1d_x6_kernel<..., P = 3>, and the shared epilogue: outputs are bit-identical
// to the 16-wave tile (tests/test_gpu_kernels.py::test_k7_tiles_large and test_h3_tiles_8_vs_16_waves, x6 cases).
#include <type_traits>

#include "bc_common.h"
#include "bc_internal.h"
#include "conv_epilogue.h"
#include "x6_common.h"

namespace bc {

constexpr int RA_MT = 6, RA_NT = 4, RA_WM = 2, RA_WN = 4, RA_NW = RA_WM * RA_WN;
constexpr int RA_BM = 16 * RA_MT * RA_WM;  // 192
constexpr int RA_BN = 16 * RA_NT * RA_WN;  // 256
constexpr int RA_QA = RA_WM * RA_MT;       // 12 m-tiles per row group (the cfg-120 / 122 packing)
constexpr int RA_APIECES = 3 * RA_QA;      // 1-KiB pieces per (chunk, tap)

// B4: 16-byte input staging (stride-1 launches with Tin % 4 == 0 and 16-B aligned rows), else single floats (also
// the phase-decomposed launches, whose rows gather the s phases of a channel)
template <bool B4>
__global__ void __launch_bounds__(512, 1) conv1d_x6ra_kernel(ConvArgs a) {
  constexpr int MT = RA_MT, NT = RA_NT, WM = RA_WM, NW = RA_NW;
  constexpr int CI = X6_MAXCOL_ITERS;                           // 32-column passes per thread (single floats)
  constexpr int NQI = 4 * NW;                                   // B4: column quads per iteration
  constexpr int IT4 = ((32 * X6_MAXCOL_ITERS + 6) / 4 + NQI - 1) / NQI;
  typedef bf16x8_t frag_t;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_ra[];

  const int ncol = a.win;
  const int bplane = a.bstage;  // bytes per B plane: ncol * 64 rounded to 16
  auto bgrp = [&](int col, int g) __attribute__((always_inline)) { return col * 64 + 16 * (g ^ ((col >> 1) & 3)); };

  const int wg = xcd_remap(blockIdx.x, a.nwg);
  const int mt_idx = wg % a.ntm;
  const int rest = wg / a.ntm;
  const int nt_idx = rest % a.ntn;
  const int b = rest / a.ntn;
  const int m0 = mt_idx * RA_BM;
  const int n0 = nt_idx * RA_BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM;
  const int wn = wave / WM;

  const unsigned long long xb_u = (unsigned long long)(a.x + (long long)b * a.xbs);
  const unsigned xb_lo = __builtin_amdgcn_readfirstlane((unsigned)xb_u);
  const unsigned xb_hi = __builtin_amdgcn_readfirstlane((unsigned)(xb_u >> 32));
  const int xbytes = __builtin_amdgcn_readfirstlane((a.ps ? a.cin0 : a.Cin) * a.Tin * 4);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long long)xb_hi << 32) | xb_lo), 0, xbytes, 0x00020000);
  const int in0 = n0 - a.pl;  // (stride 1: the phase launches run the stride-1 conv over the phases)

  const int K = a.K;
  const int nsteps = a.nchunks * K;
  // this wave's A fragments: [step][plane][12 m-tiles][64 lanes][16 B] of this row group, m-tiles wm * 6 ..; buffer
  // loads over ONE step's 36 KiB block (a resource per step: scalar base, small scalar offsets, the lane's 16 B as the
  // only vector offset; the step's offset rides in the 64-bit base, never in a large soffset)
  const unsigned long long wb_u = (unsigned long long)(reinterpret_cast<const unsigned char*>(a.w) +
                                                       (long long)mt_idx * nsteps * (RA_APIECES * 1024));
  const unsigned wb_lo = __builtin_amdgcn_readfirstlane((unsigned)wb_u);
  const unsigned wb_hi = __builtin_amdgcn_readfirstlane((unsigned)(wb_u >> 32));
  const int wlane = (wm * MT) * 1024 + lane * 16;
  auto load_a = [&](int step, int i, frag_t (&d)[3]) __attribute__((always_inline)) {
    const unsigned long long sb = (((unsigned long long)wb_hi << 32) | wb_lo) +
                                  (unsigned long long)__builtin_amdgcn_readfirstlane(step) * (RA_APIECES * 1024);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)sb, 0, RA_APIECES * 1024, 0x00020000);
#pragma unroll
    for (int q = 0; q < 3; ++q)
      d[q] = __builtin_bit_cast(frag_t, __builtin_amdgcn_raw_buffer_load_b128(wr, wlane, i * 1024 + q * RA_QA * 1024, 0));
  };

  // ---- B staging (conv1d_x6_kernel's geometry for 8 waves: the same values, the same split) ----
  const int bp = (tid >> 5) & 15;
  const int bcl = tid & 31;
  float bv0[B4 ? 1 : CI], bv1[B4 ? 1 : CI];
  auto load_b = [&](int chunk) __attribute__((always_inline)) {
    const int ci0 = chunk * X6_BKC + 2 * bp;
    int ch0 = ci0, ch1 = ci0 + 1, tb0 = in0, tb1 = in0;
    if (a.ps) {
      ch0 = ci0 / a.ps;
      ch1 = (ci0 + 1) / a.ps;
      tb0 = n0 * a.ps + (ci0 - ch0 * a.ps) - a.pl;
      tb1 = n0 * a.ps + (ci0 + 1 - ch1 * a.ps) - a.pl;
    }
    const int tstep = a.ps ? a.ps : 1;
#pragma unroll
    for (int i = 0; i < CI; ++i) {
      const int col = bcl + 32 * i;
      const int t0 = tb0 + col * tstep, t1 = tb1 + col * tstep;
      const bool cin = col < ncol;
      const unsigned o0 = (cin && ci0 < a.Cin && t0 >= 0 && t0 < a.Tin) ? (unsigned)((ch0 * a.Tin + t0) * 4) : 0xfffffff0u;
      const unsigned o1 =
          (cin && ci0 + 1 < a.Cin && t1 >= 0 && t1 < a.Tin) ? (unsigned)((ch1 * a.Tin + t1) * 4) : 0xfffffff0u;
      bv0[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o0, 0, 0));
      bv1[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, o1, 0, 0));
    }
  };
  const int r4 = ((in0 % 4) + 4) % 4;
  const int tq0 = in0 - r4;
  const int nq4 = (ncol + r4 + 3) >> 2;
  const int p4 = 8 * (wave & 1) + (lane & 7);
  const int qb4 = 8 * (wave >> 1) + (lane >> 3);
  floatx4 bq0[B4 ? IT4 : 1], bq1[B4 ? IT4 : 1];
  auto load_b4 = [&](int chunk) __attribute__((always_inline)) {
    const int c0 = chunk * X6_BKC + 2 * p4;
#pragma unroll
    for (int it = 0; it < IT4; ++it) {
      const int q = it * NQI + qb4;
      const int t = tq0 + 4 * q;
      const bool ok = q < nq4 && t >= 0 && t < a.Tin;
      const unsigned o0 = (ok && c0 < a.Cin) ? (unsigned)((c0 * a.Tin + t) * 4) : 0x80000000u;
      const unsigned o1 = (ok && c0 + 1 < a.Cin) ? (unsigned)(((c0 + 1) * a.Tin + t) * 4) : 0x80000000u;
      bq0[it] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o0, 0, 0));
      bq1[it] = __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(xr, o1, 0, 0));
    }
  };
  auto put = [&](int col, int pp, float v0, float v1, unsigned char* Bt) __attribute__((always_inline)) {
    unsigned char* p = Bt + bgrp(col, pp >> 2) + (pp & 3) * 4;
    const unsigned h = pk_bf16(v0, v1);
    const float r0 = v0 - bf_lo(h), r1 = v1 - bf_hi(h);
    const unsigned m = pk_bf16(r0, r1);
    const float s0 = r0 - bf_lo(m), s1 = r1 - bf_hi(m);
    const unsigned l = pk_bf16(s0, s1);
    *reinterpret_cast<unsigned*>(p) = h;
    *reinterpret_cast<unsigned*>(p + bplane) = m;
    *reinterpret_cast<unsigned*>(p + 2 * bplane) = l;
  };
  auto stage_load = [&](int chunk) __attribute__((always_inline)) {
    if constexpr (B4) load_b4(chunk);
    else load_b(chunk);
  };
  auto stage_store = [&](unsigned char* Bt) __attribute__((always_inline)) {
    if constexpr (B4) {
#pragma unroll
      for (int it = 0; it < IT4; ++it) {
        const int col0 = 4 * (it * NQI + qb4) - r4;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (col0 + j >= 0 && col0 + j < ncol) put(col0 + j, p4, bq0[it][j], bq1[it][j], Bt);
      }
    } else {
#pragma unroll
      for (int i = 0; i < CI; ++i) {
        const int col = bcl + 32 * i;
        if (col < ncol) put(col, bp, bv0[i], bv1[i], Bt);
      }
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  frag_t af[MT][3];  // this step's A fragments, each m-tile reloaded for the next step right after its last use
  stage_load(0);
  stage_store(smem_ra);
  if (a.nchunks > 1) stage_load(1);  // lands during chunk 0
#pragma unroll
  for (int i = 0; i < MT; ++i) load_a(0, i, af[i]);
  lds_barrier();

  const int col_lane = wn * NT * 16 + (lane & 15);
  int c = 0, tap = 0;
  // one K-step; RELOAD: request the next step's A fragments (every step but the last, which is peeled so that no
  // load is still in flight into a register when the loop ends)
  auto kstep = [&](int step, auto reload) __attribute__((always_inline)) {
    const unsigned char* Br = smem_ra + (c & 1) * 3 * bplane;
    unsigned char* Bn = smem_ra + ((c + 1) & 1) * 3 * bplane;
    const bool more = c + 1 < a.nchunks;
    const unsigned char* Bcol = Br + bgrp(col_lane + tap * a.d, lane >> 4);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      frag_t bj[3];  // (the partner wave on the SIMD covers the LDS latency: no register double buffer)
#pragma unroll
      for (int p = 0; p < 3; ++p) bj[p] = *reinterpret_cast<const frag_t*>(Bcol + j * 16 * 64 + p * bplane);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const frag_t a0 = af[i][0], a1 = af[i][1], a2 = af[i][2];
        // conv1d_x6_kernel<..., P = 3>'s chain, in its order (operands swapped: input as A)
        floatx4 t = acc[i][j];
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bj[0], a2, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bj[1], a1, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bj[2], a0, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bj[0], a1, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bj[1], a0, t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bj[0], a0, t, 0, 0, 0);
        acc[i][j] = t;
        if constexpr (decltype(reload)::value) {
          if (j == NT - 1) {  // m-tile i's fragments are dead: request step + 1's
            __builtin_amdgcn_sched_barrier(0);
            load_a(step + 1, i, af[i]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      // the next chunk's planes go into the idle buffer (last read in chunk c - 1, before the barrier that ended
      // it) in the middle of the chunk's last K-step -- their loads were issued a whole chunk ago -- and the loads of
      // chunk c + 2 go out at once into the freed registers, OLDER than every A fragment load that follows (the
      // compiler's counted waits for the A fragments then never wait for the staging loads)
      if (j == 1 && tap == K - 1 && more) {
        stage_store(Bn);
        if (c + 2 < a.nchunks) stage_load(c + 2);
      }
    }
    if (++tap == K) {
      tap = 0;
      ++c;
      lds_barrier();  // chunk c's planes stored by every wave; every wave done reading buffer (c - 1) & 1
    }
  };
  for (int step = 0; step + 1 < nsteps; ++step) kstep(step, std::true_type{});
  kstep(nsteps - 1, std::false_type{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  conv_epilogue<MT, NT>(a, acc, b, m0 + wm * MT * 16, n0 + wn * NT * 16, lane);
}

static bool x6ra_b4_fits(const ConvArgs& a) {
  return a.ps == 0 && a.s == 1 && a.Tin % 4 == 0 && a.xbs % 4 == 0 && ((unsigned long long)a.x & 15) == 0;
}

bool x6ra_applies(int K, int s, int d, int ps) {
  (void)d;
  // multi-tap stride-1 convs, the phase launches with K / s >= 2 taps, and the pointwise convs (K = 1: one K-step per
  // chunk, the next chunk's planes stored mid-step, its successor's loads a step and a half ahead; measured slower than
  // the 16-wave tile's pointwise path: C = 384 / 192 / 768 5.47 / 4.09 / 3.35 vs 4.63 / 3.45 / 3.03 ms with residual and
  // dual output, profiles/r05j_ra_pointwise.txt -- the tables keep 122 there)
  return s == 1 && (K > 1 || ps == 0);
}

const char* x6ra_kernel_name(bool b4) {
  return b4 ? "conv1d_x6ra_kernel<true>" : "conv1d_x6ra_kernel<false>";
}

// a: the conv as x6_launch prepared it (a phase-decomposed conv already rewritten as the stride-1 conv over its
// phases); w packed for a 192-row x6 tile (cfg 120 / 122).
int x6ra_launch(ConvArgs& a, int B, hipStream_t st) {
  if (a.s != 1) return BC_ERR_ARG;
  const X6Tile t{RA_MT, RA_NT, RA_WM, RA_WN};
  const int ncol = x6_ncol(t, a.K, 1, a.d);
  if (ncol > 32 * X6_MAXCOL_ITERS) return BC_ERR_UNSUPPORTED;
  a.ntm = (a.Cout + RA_BM - 1) / RA_BM;
  a.ntn = (a.Nout + RA_BN - 1) / RA_BN;
  a.nchunks = (a.Cin + X6_BKC - 1) / X6_BKC;
  a.win = ncol;
  a.bpitch = 64;
  a.bstage = (ncol * 64 + 15) / 16 * 16;
  const long long nwg = (long long)a.ntm * a.ntn * B;
  if (nwg <= 0) return BC_OK;
  if (nwg > 0x7fffffffLL) return BC_ERR_ARG;
  if ((long long)(a.ps ? a.cin0 : a.Cin) * a.Tin * 4 > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  a.nwg = (int)nwg;
  a.wsc = nullptr;
  const size_t lds = 2 * 3 * (size_t)a.bstage;
  if (lds > 160 * 1024) return BC_ERR_UNSUPPORTED;
  if (x6ra_b4_fits(a))
    hipLaunchKernelGGL(conv1d_x6ra_kernel<true>, dim3(a.nwg), dim3(512), lds, st, a);
  else
    hipLaunchKernelGGL(conv1d_x6ra_kernel<false>, dim3(a.nwg), dim3(512), lds, st, a);
  BC_CHECK_LAUNCH();
  return BC_OK;
}

}  // namespace bc

BC_DEBUG_EXPORT(conv1d_x6ra)
