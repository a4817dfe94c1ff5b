// Host logic of the x6 / h3 / bf16 conv kernels (tile selection, weight packing, launch); the kernel
// template is in conv1d_x6_kernel.h.
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
#include <algorithm>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <vector>

#include "bc_common.h"
#include "bc_internal.h"
#include "conv1d_x6_kernel.h"

namespace bc {

// cfg ids: 100 + tile (x6, three planes), 200 + tile (bf16, one plane), 300 + tile (h3, two fp16
// planes); + 1000 * s for a stride-s
// conv run by phase decomposition (ConvArgs::ps): the stride-1 conv with ceil(K/s) taps over s * Cin
// phase channels ci' = ci * s + r, weights W'[co][ci'][q] = W[co][ci][q * s + r] (0 past K).  Its
// input tile needs BN + ceil(K/s) - 1 columns instead of (BN - 1) * s + K, so the wide 128 x 256
// tile fits the stride-4/5 convs.
static inline int cfg_base(int cfg) { return cfg % 1000; }
static inline int cfg_phase(int cfg) { return cfg / 1000; }
bool x6_cfg_valid(int cfg) {
  const int b = cfg_base(cfg), s = cfg_phase(cfg);
  return ((b >= 100 && b < 100 + X6_NT) || (b >= 200 && b < 200 + X6_NT) || (b >= 300 && b < 300 + X6_NT)) &&
         (s == 0 || (s >= 2 && s <= 16));
}
// 100..: x6 (3 bf16 planes), 200..: bf16 (1 plane), 300..: h3 (2 fp16 planes + per-row scales)
static inline int cfg_planes(int cfg) {
  const int b = cfg_base(cfg);
  return b >= 300 ? 2 : b >= 200 ? 1 : 3;
}
static inline int planes_base(int planes) { return planes == 1 ? 200 : planes == 2 ? 300 : 100; }
static inline const X6Tile& cfg_tile(int cfg) { return kX6Tiles[cfg_base(cfg) % 100]; }
const X6Tile& x6_tile(int cfg) { return cfg_tile(cfg); }

// Returns a x6 (planes = 3) / bf16 (planes = 1) cfg id, or -1 when the shape should stay on the
// fp32 kernel.
// Two-workgroup-per-CU preference: NT == 1 tiles whose LDS fits twice in a CU let one workgroup's
// operand loads and epilogue stores overlap the other's MFMAs.  Measured on MI355X (profiles/
// r01_occ_sweep.txt): a win for the short-K / small-M convs (Cout <= 384 with Cin*K <= 1536: the
// C = 192 k7 and k1 convs, the C = 384 k1 conv, the stride-2 convs), a loss for the long-K ones.
// BC_X6_OCC (tuning experiments): 4 = always try them first, 2 = never, unset = that rule.
static int x6_occ_pref() {
  static int v = [] {
    const char* e = getenv("BC_X6_OCC");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static int x6_select_tile(int Cout, int Cin, int K, int s, int d, int planes);

// Stride >= 3 convs with dilation 1 (the encoder's k=2s downsampling) run phase-decomposed
// (BC_X6_PHASE=0 disables it for A/B timing).
static bool x6_phase_ok(int s, int d) {
  static int v = [] {
    const char* e = getenv("BC_X6_PHASE");
    return e ? atoi(e) : 1;
  }();
  return v && s >= 3 && s <= 16 && d == 1;
}

// Measured tile preferences of the x6 (three-plane) kernel, from a sweep of every tile over the
// BigCodec encoder's conv shapes (tools/conv_bench.py --cfg all, profiles/r01_tile_sweep.txt):
//   pointwise, Cout % 128 == 0     -> 101 (128 x 128, two-chunk B prefetch): C = 384 / 768 and the
//                                     LSTM input projection 1536 -> 6144, 12-24 % under the others
//   pointwise, Cout % 96 == 0      -> 116 (96 x 64, two workgroups per CU): C = 192
//   stride 1, K > 1, Cout % 96 == 0 and <= 384 -> 109 (96 x 128, all 8 waves on one 96-row block,
//                                     two workgroups per CU): k7 C = 192 -17 %, C = 384 -2 %
//   stride 2, Cout % 96 == 0 and <= 192 -> phase-decomposed 109: the k4 downsampling at C = 48 / 96
//                                     -33 % / -7 %
// Returns the cfg or -1 (then the general rules below decide).
static int x6_preferred_cfg(int Cout, int Cin, int K, int s, int d) {
  auto fits2 = [](int tile, int K_, int s_, int d_) {  // two workgroups per CU: LDS <= 80 KiB
    const X6Tile& t = kX6Tiles[tile];
    const int ncol = x6_ncol(t, K_, s_, d_);
    return ncol <= 32 * X6_MAXCOL_ITERS && x6_lds(t, ncol, 3, s_) <= 80 * 1024;
  };
  if (s == 1 && K == 1) {
    if (Cout % 128 == 0) return 101;
    if (Cout % 96 == 0) return 116;
    return -1;
  }
  if (s == 1 && Cout % 96 == 0 && Cout <= 384 && fits2(9, K, 1, d)) return 109;
  if (s == 2 && d == 1 && Cout % 96 == 0 && Cout <= 192 && Cin * 2 >= 32 && fits2(9, (K + 1) / 2, 1, 1))
    return 2000 + 109;
  return -1;
}

// Measured tile preferences of the h3 (two-plane) kernel (tools/tile_sweep.sh, tools/x6_tile_sweep2.sh /
// 3.sh; profiles/r01f_h3_tile_sweep.txt, r01g_wide_tile_sweep*.txt), where they differ from the x6 ones:
//   stride 1, K > 1, Cout % 192 == 0 -> 120 (192 x 256, 96 x 64 per wave, two taps per K-step):
//                                     k7 C = 192 / 384 -9 / -14 % vs 109, decoder k7 1024 -> 1536 -8 %
//   stride 1, K > 1, Cout == 768 or Cout % 256 == 0 (not % 192) -> 121 (256 x 256): k7 C = 768 -16 %,
//                                     the final k3 1536 -> 1024 -16 %
//   stride >= 3, d = 1, Cout % 256 == 0 -> phase-decomposed 121: the stride-5 downsampling convs -9..-14 %
//                                     vs the direct strided 256 x 64 tile
//   pointwise, Cout % 192 == 0     -> 114 (192 x 128): C = 192 / 384 / 768, 10-20 % under 101 / 116
//                                     (the x256 tiles lose 20-30 % here), except Cout >= 2048 with
//                                     Cout % 256 == 0 (the LSTM input projection) -> 121
//   stride 2, Cout % 192 == 0 and <= 384 -> 115 (192 x 64, direct strided B tile): -15 %; except
//                                     Cout % 384 == 0 -> phase-decomposed 120: 192 -> 384 -3.5 %
//   stride >= 3, d = 1, Cout % 192 == 0 -> phase-decomposed 120 (two taps per K-step fit, 121 runs
//                                     one): the stride-5 downsampling 384 -> 768 / 768 -> 1536 -3 / -7 %
//                                     vs phase-decomposed 121 (profiles/r02_s2_sweep.txt)
// The 16-wave (1024-thread) 192 x 256 tile 122 (96 x 32 per wave) by shape class, a bit each
// (BC_X6_W16 overrides the mask for A/B timing):
//   1: stride-1 multi-tap convs with Cout % 192 == 0 instead of the 8-wave 120
//   2: the phase-decomposed strided convs with Cout % 192 == 0 instead of 120
//   4: the k7 C = 768 convs instead of the 256 x 256 tile 121
//   8: the pointwise C = 192 convs instead of 114 (off by default since the 16-byte staging: 114 2.99 vs 3.08 ms in
//      h3 and 2.70 vs 2.78 in bf16 with residual + dual output, profiles/r04j_pw_tiles.txt)
//  16: the pointwise Cout >= 2048 convs (the LSTM input projection) instead of the 256 x 256 tile 121
static int x6_w16() {
  static const int v = [] {
    const char* e = getenv("BC_X6_W16");
    return e ? atoi(e) : 23;
  }();
  return v;
}
static int w16(int bit, int tile8, int tile16) { return (x6_w16() & bit) ? tile16 : tile8; }

static int h3_preferred_cfg(int Cout, int Cin, int K, int s, int d) {
  (void)Cin;
  // Cout = 1 (the decoder's last conv, 48 -> 1, k7): the 16 x 256 tile (two taps per K-step over the double B buffer)
  // instead of the 16 x 128 two-per-CU tile 113: half the workgroups of a conv with one output row, 2.83 -> 1.73 ms at
  // B = 64 x 240 000 (profiles/r03y_cout1.txt)
  if (Cout == 1 && s == 1 && x6_ncol(kX6Tiles[8], K, 1, d) <= 32 * X6_MAXCOL_ITERS) return 108;
  if (s == 1 && K == 1) {
    if (Cout >= 2048 && Cout % 192 == 0 && (x6_w16() & 16)) return 122;
    if (Cout >= 2048 && Cout % 256 == 0) return 121;
    if (Cout % 192 == 0) return Cout == 192 ? w16(8, 114, 122) : 114;
  }
  if (s == 1 && K > 1) {
    const bool f320 = Cout % 192 == 0, f321 = Cout % 256 == 0;
    auto fits = [&](int tile) { return x6_ncol(kX6Tiles[tile], K, 1, d) <= 32 * X6_MAXCOL_ITERS; };
    if (Cout == 768 && (x6_w16() & 4) && fits(22)) return 122;
    if ((Cout == 768 || (f321 && !f320)) && fits(21)) return 121;
    if (f320 && fits(20)) return w16(1, 120, 122);
  }
  auto phase_fits = [&](int tile) {
    return x6_ncol(kX6Tiles[tile], (K + s - 1) / s, 1, 1) <= 32 * X6_MAXCOL_ITERS;
  };
  if (s == 2 && d == 1 && Cout % 384 == 0 && phase_fits(20)) return 2000 + w16(2, 120, 122);
  // 96 -> 192: 3.39 -> 2.69 ms on the phase-decomposed 16-wave tile (profiles/r02h_s2_w16.txt; 48 -> 96, a
  // half-empty 192-row tile, stays on 109)
  if (s == 2 && d == 1 && Cout % 192 == 0 && (x6_w16() & 2) && phase_fits(22)) return 2000 + 122;
  if (s == 2 && d == 1 && Cout % 192 == 0 && Cout <= 384) return 115;
  if (s >= 3 && s <= 16 && d == 1 && Cout % 192 == 0 && phase_fits(20)) return 1000 * s + w16(2, 120, 122);
  if (s >= 3 && s <= 16 && d == 1 && Cout % 256 == 0 && x6_ncol(kX6Tiles[21], (K + s - 1) / s, 1, 1) <= 32 * X6_MAXCOL_ITERS)
    return 1000 * s + 121;
  if (s >= 3 && d == 1 && Cout % 256 == 0 && x6_ncol(kX6Tiles[2], K, s, d) <= 32 * X6_MAXCOL_ITERS) return 102;
  return -1;
}

// Measured x6 (three-plane) preferences of round 4 (tools/x6_table_sweep.sh, profiles/r04c_x6_sweep.txt, B = 64 x 10 s
// encoder shapes), where the round-1 table above loses: the 16-wave 192 x 256 tile (x6 without the A-fragment prefetch,
// 16-byte input staging on stride-1 launches) on every Cout % 192 == 0 conv -- k7 C = 192 / 384 / 768 10.18 / 19.55 /
// 13.83 -> 8.95 / 16.34 / 12.79 ms, pointwise C = 192 / 384 / 768 3.79 / 4.95 / 3.47 -> 3.31 / 4.67 / 3.19, the LSTM
// input projection 8.99 -> 7.89, phase-decomposed stride 2 96 -> 192 / 192 -> 384 4.86 / 8.05 -> 3.97 / 6.44, stride 5
// 768 -> 1536 10.79 -> 8.96 -- except the stride-5 384 -> 768 (phase-decomposed 256 x 256: 13.58 -> 10.94) and the final
// k3 1536 -> 1024 (256 x 256: 4.02 -> 3.59); 48 -> 96 stride 2 keeps the 96-row tile (2109: 3.16 vs 4.89).
// BC_X6_RA (bits; default 2): the register-A kernel (conv1d_x6ra.hip, x6 on the 8-wave 192 x 256 tile = cfg 120) for
// 1: the multi-tap stride-1 convs with Cout % 192 == 0, 2: the phase-decomposed stride >= 3 ones, in place of the
// 16-wave tile 122 (same packing, bit-identical outputs).  Measured (profiles/r05g_ra.txt, B = 64): stride 5 384 -> 768
// 10.61 -> 10.46 ms, 768 -> 1536 8.67 -> 8.38; the k7 convs 8.55 -> 9.08 (C = 192 d9), 15.66 -> 16.06 (384), 12.28 ->
// 12.19 (768) and the stride-2 phase convs 6.36 -> 6.91, 4.05 -> 4.66 stay on 122.
static int x6_ra() {
  static const int v = [] {
    const char* e = getenv("BC_X6_RA");
    return e ? atoi(e) : 2;
  }();
  return v;
}

static int x6p3_preferred_cfg(int Cout, int Cin, int K, int s, int d) {
  (void)Cin;
  auto fits = [&](int tile, int K_, int s_, int d_) { return x6_ncol(kX6Tiles[tile], K_, s_, d_) <= 32 * X6_MAXCOL_ITERS; };
  const int ra1 = (x6_ra() & 1) ? 120 : 122, ra2 = (x6_ra() & 2) ? 120 : 122;
  if (s == 1 && K > 1 && Cout % 192 == 0 && fits(22, K, 1, d)) return ra1;
  if (s == 1 && Cout % 192 == 0 && fits(22, K, 1, d)) return 122;
  if (s == 1 && K > 1 && Cout % 256 == 0 && fits(21, K, 1, d)) return 121;
  const int Kp = (K + s - 1) / s;
  if (s == 2 && d == 1 && Cout % 192 == 0 && fits(22, Kp, 1, 1)) return 2000 + 122;
  if (s >= 3 && s <= 16 && d == 1) {
    // (the register-A tile also beats the 256 x 256 one at 384 -> 768: 10.83 -> 10.39 ms, profiles/r05w_strided.txt)
    if (Cout % 192 == 0 && (Cout >= 1536 || (ra2 == 120 && Kp > 1)) && fits(22, Kp, 1, 1))
      return 1000 * s + (Kp > 1 ? ra2 : 122);
    if (Cout % 256 == 0 && fits(21, Kp, 1, 1)) return 1000 * s + 121;
    if (Cout % 192 == 0 && fits(22, Kp, 1, 1)) return 1000 * s + (Kp > 1 ? ra2 : 122);
  }
  return -1;
}

// BC_X6_TABLE=1 restores the round-1 x6 table (A/B timing).
static bool x6_table_r4() {
  static const bool v = [] {
    const char* e = getenv("BC_X6_TABLE");
    return !e || atoi(e) != 1;
  }();
  return v;
}

int x6_select_cfg(int Cout, int Cin, int K, int s, int d, int planes) {
  if (Cin < 16) return -1;  // e.g. the first conv (Cin = 1): no K to amortise the split over
  if (planes == 3 && x6_occ_pref() == 0 && x6_table_r4()) {
    const int c = x6p3_preferred_cfg(Cout, Cin, K, s, d);
    if (c >= 0) return c;
  }
  if (planes <= 2 && x6_occ_pref() == 0) {  // bf16 (1 plane) follows the h3 table (measured, config 5)
    const int c = h3_preferred_cfg(Cout, Cin, K, s, d);
    if (c >= 0) return c + (planes == 2 ? 200 : 100);  // (a phase-decomposed 1000 * s + tile keeps its phase factor)
  }
  if (planes >= 2 && x6_occ_pref() == 0) {
    const int c = x6_preferred_cfg(Cout, Cin, K, s, d);
    if (c >= 0) return c + (planes == 2 ? 200 : 0);
  }
  if (x6_phase_ok(s, d)) {
    const int c = x6_select_tile(Cout, Cin * s, (K + s - 1) / s, 1, 1, planes);
    if (c >= 0) return 1000 * s + c;
  }
  return x6_select_tile(Cout, Cin, K, s, d, planes);
}

// Narrow launches (a stream's chunk, a small batch): the shape tables above assume thousands of output columns per
// clip.  The 16-wave 192 x 256 tile computes 256 columns per clip whatever Tout is, so a stride-1 multi-tap conv (or a
// phase-decomposed strided one, whose phase conv has K / s taps) with Tout <= 128 moves to a tile whose width covers
// Tout (64 or 128 columns), and to fewer rows (96 / 32) when 192-row tiles would leave the CUs idle; a pointwise conv
// takes a 64-column tile up to 128 columns.  Measured on five k7 and four pointwise stream / small-batch shapes: the
// rule picks the fastest tile on each, 1.3-2.5x per k7 launch, 1.1-2.2x per pointwise one
// (profiles/r04s_narrow_sweep.txt, r04u_pw_narrow_sweep.txt).  Same K order per output: x6 and bf16 results do not
// depend on the tile; h3's block scales follow the staged tile (fp32 rounding level).  BC_X6_NARROW=0 disables it.
int x6_narrow_cfg(int cfg, int Cout, int K, int s, int d, int planes, int B, int Tout, int cus) {
  static const bool on = [] {
    const char* e = getenv("BC_X6_NARROW");
    return !(e && atoi(e) == 0);
  }();
  const int base = planes == 3 ? 0 : planes == 1 ? 100 : 200;
  if (cfg >= 1000) {  // a phase-decomposed strided conv: the stride-1 conv over ps phase rows per channel
    const int ps = cfg / 1000;
    if (s != ps || d != 1) return cfg;
    const int inner = x6_narrow_cfg(cfg % 1000, Cout, (K + s - 1) / s, 1, 1, planes, B, Tout, cus);
    return 1000 * ps + inner;
  }
  if (!on || s != 1 || Tout > 128 || Tout <= 0 || B <= 0) return cfg;
  if (K == 1) {  // pointwise: 64-column tiles win up to 128 columns (two n-tiles per clip), 192 rows when they fill
    if (cfg - base != 114 && cfg - base != 122) return cfg;
    const long long n192 = (long long)((Cout + 191) / 192) * ((Tout + 63) / 64) * B;
    const int tile = (Cout % 192 == 0 && n192 >= cus) ? 15 : (Cout % 96 == 0 ? 16 : -1);
    return tile < 0 ? cfg : base + 100 + tile;
  }
  int tile;
  if (cfg - base == 121) {  // the 256 x 256 tile (Cout % 256 == 0, e.g. the encoder's final k3): 128 x 64 up to 64
    if (Tout > 64 || Cout % 128 != 0) return cfg;  // columns (k3 1536 -> 1024: 0.377 -> 0.176 ms at 16 x 6 columns,
    tile = 17;                                      // 0.411 -> 0.245 at 64 x 24; profiles/r04y_k3_sweep.txt)
  } else {
    // (x6: the register-A tile 120 narrows like 122; h3's block scales follow the tile, so its 320 stays)
    if (cfg - base != 122 && !(planes == 3 && cfg - base == 120)) return cfg;
    auto nwg = [&](int bm) { return (long long)((Cout + bm - 1) / bm) * B; };
    const bool fill192 = Cout % 192 == 0 && nwg(192) >= cus;
    if (Tout <= 64) tile = fill192 ? 15 : (Cout % 96 == 0 ? 16 : 12);
    else tile = fill192 ? 14 : 12;
  }
  if (x6_ncol(kX6Tiles[tile], K, 1, d) > 32 * X6_MAXCOL_ITERS) return cfg;
  return base + 100 + tile;
}

static int x6_select_tile(int Cout, int Cin, int K, int s, int d, int planes) {
  int order[8];
  bool occ4[8] = {false};
  int n = 0;
  const int pref = x6_occ_pref();
  if (pref == 4 || (pref == 0 && Cout <= 384 && Cin * K <= 1536)) {
    int c = -1;
    if (Cout >= 128) c = Cout % 128 == 0 ? 17 : Cout % 96 == 0 ? 16 : -1;
    else {
      const int mt = (Cout + 15) / 16;
      c = mt >= 5 ? 9 : mt == 4 ? 10 : mt == 3 ? 11 : mt == 2 ? 12 : 13;
    }
    if (c >= 0) {
      occ4[n] = true;
      order[n++] = c;
    }
  }
  if (Cout >= 128 && Cout % 128 != 0 && Cout % 192 == 0) {
    // 192-row tiles: no half-empty m-tile at C = 192 / 576
    if (s <= 2) order[n++] = 14;
    order[n++] = 15;
  }
  if (Cout >= 128) {
    if (s == 1) order[n++] = 0;
    if (s <= 2) order[n++] = 1;
    if (Cout >= 256) order[n++] = 2;
    order[n++] = 3;
  } else {
    const int mt = (Cout + 15) / 16;
    const int base = mt == 6 || mt == 5 ? 0 : mt == 4 ? 1 : mt == 3 ? 2 : mt == 2 ? 3 : 4;
    if (mt > 6) return -1;
    order[n++] = 4 + base;
    order[n++] = 9 + base;
  }
  for (int i = 0; i < n; ++i) {
    const X6Tile& t = kX6Tiles[order[i]];
    const int ncol = x6_ncol(t, K, s, d);
    if (ncol > 32 * X6_MAXCOL_ITERS) continue;
    if (x6_lds(t, ncol, planes, s) > (occ4[i] ? 80 : 160) * 1024) continue;
    return planes_base(planes) + order[i];
  }
  return -1;
}

long long x6_packed_bytes(int Cout, int Cin, int K, int cfg) {
  const X6Tile& t = cfg_tile(cfg);
  if (const int s = cfg_phase(cfg)) {
    Cin *= s;
    K = (K + s - 1) / s;
  }
  const int ntm = (Cout + x6_BM(t) - 1) / x6_BM(t);
  const int nchunks = (Cin + X6_BKC - 1) / X6_BKC;
  const long long planes = (long long)ntm * nchunks * K * cfg_planes(cfg) * t.WM * t.MT * 1024;
  return planes + (cfg_planes(cfg) == 2 ? (long long)ntm * x6_BM(t) * 4 : 0);  // h3: + 1 / row scale
}

static inline unsigned short f2bf_rn(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);  // NaN
  const unsigned r = u + 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(r >> 16);
}
static inline unsigned short f2h_rn(float f) {
  const _Float16 h = (_Float16)f;  // IEEE round-to-nearest-even
  unsigned short u;
  memcpy(&u, &h, 2);
  return u;
}
static inline float h2f(unsigned short u) {
  _Float16 h;
  memcpy(&h, &u, 2);
  return (float)h;
}
static inline float bf2f(unsigned short h) {
  const unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// w: [Cout][Cin][K] fp32 host -> packed bf16 planes (host), layout documented at the top.
void x6_pack_weight(const float* w, unsigned short* out, int Cout, int Cin, int K, int cfg) {
  if (const int s = cfg_phase(cfg)) {  // phase-decomposed weights W'[co][ci * s + r][q]
    const int Kp = (K + s - 1) / s, Cp = Cin * s;
    std::vector<float> wp((size_t)Cout * Cp * Kp, 0.f);
    for (int co = 0; co < Cout; ++co)
      for (int ci = 0; ci < Cin; ++ci)
        for (int k = 0; k < K; ++k)
          wp[((size_t)co * Cp + ci * s + k % s) * Kp + k / s] = w[((size_t)co * Cin + ci) * K + k];
    x6_pack_weight(wp.data(), out, Cout, Cp, Kp, cfg_base(cfg));
    return;
  }
  const X6Tile& t = cfg_tile(cfg);
  const int P = cfg_planes(cfg);
  const int BM = x6_BM(t), QA = t.WM * t.MT;
  const int ntm = (Cout + BM - 1) / BM;
  const int nchunks = (Cin + X6_BKC - 1) / X6_BKC;
  // h3: per-row power-of-two scale 2^(14 - e), 2^e <= max |w[row]| < 2^(e+1) (see x6_common.h)
  std::vector<float> rsc(P == 2 ? (size_t)ntm * BM : 0, 1.f);
  for (size_t row = 0; row < rsc.size() && (int)row < Cout; ++row) {
    float m = 0.f;
    for (long long k = 0; k < (long long)Cin * K; ++k) m = std::max(m, std::fabs(w[(long long)row * Cin * K + k]));
    if (m > 0.f && std::isfinite(m)) {
      const int e = std::max(-112, std::min(140, std::ilogb(m)));
      rsc[row] = std::ldexp(1.f, 14 - e);
    }
  }
  long long o = 0;
  for (int mg = 0; mg < ntm; ++mg)
    for (int c = 0; c < nchunks; ++c)
      for (int tap = 0; tap < K; ++tap)
        for (int p = 0; p < P; ++p)
          for (int q = 0; q < QA; ++q)
            for (int lane = 0; lane < 64; ++lane)
              for (int j = 0; j < 8; ++j, ++o) {
                const int row = mg * BM + q * 16 + (lane & 15);
                const int ci = c * X6_BKC + 8 * (lane >> 4) + j;
                float v = 0.f;
                if (row < Cout && ci < Cin) v = w[((long long)row * Cin + ci) * K + tap];
                if (P == 2) {
                  const float vs = v * rsc[row];
                  const unsigned short g0 = f2h_rn(vs);
                  out[o] = p == 0 ? g0 : f2h_rn(vs - h2f(g0));
                  continue;
                }
                const unsigned short h0 = f2bf_rn(v);
                const float r1 = v - bf2f(h0);
                const unsigned short h1 = f2bf_rn(r1);
                const float r2 = r1 - bf2f(h1);
                const unsigned short h2 = f2bf_rn(r2);
                out[o] = p == 0 ? h0 : p == 1 ? h1 : h2;
              }
  if (P == 2) {  // 1 / row scale after the planes (ConvArgs::wsc)
    float* inv = reinterpret_cast<float*>(out + o);
    for (size_t row = 0; row < rsc.size(); ++row) inv[row] = 1.f / rsc[row];
  }
}

int x6_kernel_name(int cfg, int K, int s, int d, char* buf, int n) {
  if (!x6_cfg_valid(cfg)) return -1;
  if (const int ps = cfg_phase(cfg)) {  // the stride-1 conv over the phases (x6_launch)
    K = (K + ps - 1) / ps;
    s = d = 1;
  }
  const X6Tile& t = cfg_tile(cfg);
  const int P = cfg_planes(cfg);
  if (P == 3 && cfg_base(cfg) == 120 && x6ra_applies(K, s, d, cfg_phase(cfg)))  // x6_launch's routing
    return snprintf(buf, n, "%s", x6ra_kernel_name(cfg_phase(cfg) == 0));
  const X6Variant v = x6_variant(t, P, K, s, d, cfg_phase(cfg));
  // (the 16-byte staging also needs Tin % 4 == 0 and 16-B aligned rows at launch, x6_b4_fits: true of every
  // BigCodec shape at the configs' clip lengths; a launch that fails it runs the single-float variant)
  const int T4 = P == 1 ? 4 : P == 2 ? 2 : 1;
  const bool b4 = v.b4 && (v.pw || (v.tps == T4 && v.db == (P == 1)));
  return snprintf(buf, n, "conv1d_x6_kernel<%d, %d, %d, %d, %d, %s, %d, %s, %s>", t.MT, t.NT, t.WM, t.WN, P,
                  v.pw ? "true" : "false", v.tps, v.db ? "true" : "false", b4 ? "true" : "false");
}

int x6_launch(ConvArgs& a, int B, int cfg, hipStream_t st) {
  static const int dbg = [] {
    const char* e = getenv("BC_X6_DEBUG");
    return e ? atoi(e) : 0;
  }();
  a.dbg = dbg;
  a.ps = 0;
  if (const int s = cfg_phase(cfg)) {  // run as the stride-1 conv over the s phases
    if (a.s != s || a.d != 1 || a.ostride != 1) return BC_ERR_ARG;
    a.ps = s;
    a.cin0 = a.Cin;
    a.Cin *= s;
    a.K = (a.K + s - 1) / s;
    a.s = 1;
    cfg = cfg_base(cfg);
  }
  const int tile = cfg_base(cfg) % 100;
  if (cfg_planes(cfg) == 3 && tile == 20 && x6ra_applies(a.K, a.s, a.d, a.ps)) return x6ra_launch(a, B, st);
  switch (cfg_planes(cfg)) {
    case 1: return x6_launch_tile<1>(a, B, tile, st);
    case 2: return x6_launch_tile<2>(a, B, tile, st);
    case 3: return x6_launch_tile<3>(a, B, tile, st);
  }
  return BC_ERR_ARG;
}

}  // namespace bc
