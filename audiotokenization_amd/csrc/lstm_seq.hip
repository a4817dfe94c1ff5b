// Persistent ResLSTM recurrence (vq/module.py:143-167 -> torch.nn.LSTM, batch_first,
// unidirectional): ONE launch per layer walks all T steps.
//
// Why persistent: one step of the default model (H = 1536, 64 clips) is a 6144 x 1536 x 64 GEMM
// plus the cell update.  As one launch per step (lstm.hip) every step re-reads W_hh (37.7 MB) from
// the Infinity Cache and pays a kernel boundary.  Here every workgroup keeps its slice of W_hh in
// VGPRs for the whole sequence; the only per-step traffic is h_{t-1} (H x 64 fp32, read by every
// workgroup from L2) and a per-workgroup flag.
//
// Geometry: G = H / 8 workgroups (192 for H = 1536, one per CU, all co-resident), 256 threads.
//   workgroup g owns hidden units 8g..8g+7 = 32 gate rows = two 16-row m-tiles whose rows are
//   unit-major (m = 4*unit + gate), so after the MFMA a lane holds the i,f,g,o pre-activations of
//   one (unit, clip) cell in its four accumulator registers.
//   wave w owns K = [w*H/4, (w+1)*H/4): KS = H/128 k-steps of 32; its W_hh fragments (2 m-tiles x
//   KS x 3 bf16 planes) are loaded once.
// Arithmetic: the fp32-accurate 3xbf16 split of conv1d_x6.hip (six bf16 MFMAs per product term);
//   h is split on the fly, W_hh on the host.  The four waves' partial sums are reduced through LDS
//   in a fixed order, then c = f*c + i*g, h = o*tanh(c) with c held in registers.
// Hand-off of h_t: the workgroup gathers its 8 units x 64 clips in LDS, one wave splits them into
//   the three bf16 planes and writes them with 16-byte write-through (sc1) stores into slot t of the
//   fragment-native sequence buffer hseq[t][k-step][n-tile][plane][lane][8 bf16] (the consumers'
//   MFMA B fragments as they are), drains them (vmcnt(0)) and one lane stores flags[g] = t+1
//   (relaxed, agent scope).  Consumer wave w polls the flags of the G/4 workgroups that produce its
//   K range (sc1 loads, bounded spin), then reads slot t-1 with 16-byte sc1 buffer loads
//   (ls_load_sc1).  That is the measured-valid hand-off of MI355X_MICROARCH.md (§Workgroup dispatch,
//   "Valid forms", table row 1: sc1 payload stores, vmcnt(0), one lane's sc1 flag store; sc1 poll;
//   EVERY load of the handed-off bytes an sc1 load).  Rounds 1-2 read the slot with PLAIN loads and
//   no agent-scope acquire, arguing that a slot written once per launch cannot be cached stale; the
//   guide lists exactly that form as invalid ("no acquire -> stale, first touch included"), and
//   it is the one cross-workgroup hand-off of the x6 full-size path whose visibility was not
//   guaranteed (x6 latent 5.1e-4 off on one box).  sc1 loads bypass
//   only the CU's L1; the XCD's L2 still serves its CUs.
//   Every poll is bounded: on timeout the kernel counts it in *status and all workgroups leave.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bc_common.h"
#include "bc_internal.h"
#include "x6_common.h"

namespace bc {

typedef __bf16 ls_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 ls_bf16x2 __attribute__((ext_vector_type(2)));
typedef float ls_float2 __attribute__((ext_vector_type(2)));
typedef unsigned ls_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned ls_gu32;

constexpr int LS_U = 8;          // hidden units per workgroup
constexpr int LS_WAVES = 4;
constexpr int LS_NB = 64;        // clips per launch (4 n-tiles of 16)
constexpr int LS_HD = 4;         // lstm_seq2: depth of the h_{t-1} register ring (k-steps)
constexpr int LS_HSTEP_PER_UNIT = LS_NB * 3 / 2;  // floats of hseq per hidden unit per step (3 bf16 planes)
constexpr int LS_SC1 = 16;       // buffer-op cache policy: sc1 (write-through / L1 bypass)
constexpr unsigned LS_SPIN_LIMIT = 1u << 22;
constexpr int LS_FLAG_BYTES = 2 * 256 * 4;  // flags[half][workgroup], G <= 256

struct LstmSeqArgs {
  const float* gx;            // [4H][T*Btot] input projection incl. b_ih + b_hh (ctb layout)
  const unsigned short* whh;  // lstm_seq_pack layout
  float* y;                   // [H][T*Btot] output h_t (ctb layout)
  float* hseq;                // [T][H/32][4][64][8] fp32: h_t in MFMA-fragment order, one slot per step
  unsigned* flags;            // [G], zero before the launch
  int* status;                // this call's timeout counter (0 = ok), zeroed by the caller on the stream
  int* status_total;          // process-wide diagnostic counter (bc_lstm_status)
  unsigned spin_limit;        // polls before a workgroup gives up (LS_SPIN_LIMIT; tests force a small one)
  int H, T, Btot, b0, nb;
  int dbg;  // timing experiments only (BC_LSTM_SEQ_DEBUG): 4 = skip the flag poll (wrong results)
  long long* stamps;  // diagnostic s_memtime stamps (BC_LSTM_SEQ_STAMPS), nullptr in normal runs
  // carried state (lstm_seq2 only; streaming): h0 / c0 [H][Btot] initial state or nullptr (zeros);
  // hT / cT [H][Btot] final state or nullptr.  With h0, hseq slot 0 holds h0 and step t's h_t is
  // published to slot t + 1 (flag t + 2).
  const float* h0;
  const float* c0;
  float* hT;
  float* cT;
};

constexpr int LS_STAMP_T = 2048;  // steps recorded per stamped workgroup

template <int P> struct LsFrag { typedef __bf16 type __attribute__((ext_vector_type(8))); };
template <> struct LsFrag<2> { typedef _Float16 type __attribute__((ext_vector_type(8))); };

__device__ __forceinline__ unsigned ls_pk(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((ls_float2){a, b}, ls_bf16x2));
}

// split 8 fp32 values into three bf16x8 planes, v = p0 + p1 + p2 exactly
__device__ __forceinline__ void ls_split8(const float (&v)[8], ls_bf16x8 (&p)[3]) {
  unsigned h[4], m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = v[2 * i], b = v[2 * i + 1];
    h[i] = ls_pk(a, b);
    const float ra = a - __uint_as_float(h[i] << 16), rb = b - __uint_as_float(h[i] & 0xffff0000u);
    m[i] = ls_pk(ra, rb);
    const float sa = ra - __uint_as_float(m[i] << 16), sb = rb - __uint_as_float(m[i] & 0xffff0000u);
    l[i] = ls_pk(sa, sb);
  }
  p[0] = __builtin_bit_cast(ls_bf16x8, (ls_u32x4){h[0], h[1], h[2], h[3]});
  p[1] = __builtin_bit_cast(ls_bf16x8, (ls_u32x4){m[0], m[1], m[2], m[3]});
  p[2] = __builtin_bit_cast(ls_bf16x8, (ls_u32x4){l[0], l[1], l[2], l[3]});
}

// Cell nonlinearities on the hardware exp / reciprocal (v_exp_f32, v_rcp_f32: ~1 ulp each): the
// OCML expf / division / tanhf versions took 2200 of a step's 30 000 cycles (stamped timeline,
// tools/lstm_bench.py).  tanh(x) = 1 - 2 / (1 + e^{2x}) saturates exactly to +-1 and has an absolute
// error ~1e-7 near 0, the fp32-class error the recurrence test bounds.
__device__ __forceinline__ float ls_sigmoid(float x) { return __frcp_rn(1.0f + __expf(-x)); }
__device__ __forceinline__ float ls_tanh(float x) { return 1.0f - 2.0f * __frcp_rn(1.0f + __expf(2.0f * x)); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ls_rsrc(const void* p, unsigned bytes) {
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0,
                                           __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// 16-byte sc1 load of a handed-off h_t fragment (L1 bypass: see the hand-off notes at the top)
template <typename T>
__device__ __forceinline__ T ls_load_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  static_assert(sizeof(T) == 16, "16-byte fragments");
  return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, LS_SC1));
}

template <int KS>
__global__ void __launch_bounds__(256, 1) lstm_seq_x6_kernel(LstmSeqArgs a) {
  __shared__ floatx4 red[LS_WAVES][8][64];  // per-wave partial gates of the 8 (m-tile, n-tile) tiles
  __shared__ float hs[LS_NB][LS_U + 1];     // h_t gathered per clip
  __shared__ int bail;

  const int g = blockIdx.x;
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H;
  const long long TB = (long long)a.T * a.Btot;
  if (tid == 0) bail = 0;

  // ---- W_hh slice -> registers (once) ----
  ls_bf16x8 wr[2][KS][3];
  {
    const ls_bf16x8* wp = reinterpret_cast<const ls_bf16x8*>(a.whh) + (long long)(g * LS_WAVES + w) * (2 * KS * 3) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int p = 0; p < 3; ++p) wr[mt][ks][p] = wp[((mt * KS + ks) * 3 + p) * 64];
  }

  // cells of this thread: tiles p = 2w + q (q = 0, 1); m-tile p>>2, n-tile p&3
  int cu[2], cb[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = 2 * w + q;
    cu[q] = (p >> 2) * 4 + (lane >> 4);  // unit within the workgroup
    cb[q] = (p & 3) * 16 + (lane & 15);  // clip within the launch
  }
  float cst[2] = {0.f, 0.f};

  const long long hstep = (long long)H * LS_HSTEP_PER_UNIT;  // floats of hseq per step
  const int nprod = G / LS_WAVES;                // producers of this wave's K range
  ls_gu32* flags = (ls_gu32*)(a.flags);

  // input-projection gates of my two cells (independent of the recurrence: prefetched a step ahead)
  auto load_gx = [&](int t, float (&dst)[2][4]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int unit = g * LS_U + cu[q];
      const bool ok = cb[q] < a.nb;
#pragma unroll
      for (int gate = 0; gate < 4; ++gate)
        dst[q][gate] = ok ? a.gx[((long long)gate * H + unit) * TB + (long long)t * a.Btot + a.b0 + cb[q]] : 0.f;
    }
  };
  float gxv[2][4], gxn[2][4];
  load_gx(0, gxv);

  // diagnostic timeline of workgroups 0 and G/2: [wg][t][wave][event]
  long long* stamp_row = nullptr;
  if (a.stamps && lane == 0 && (g == 0 || g == G / 2)) stamp_row = a.stamps + (long long)(g == 0 ? 0 : 1) * LS_STAMP_T * 32;
#define LS_STAMP(ev)                                                                             \
  if (stamp_row && t < LS_STAMP_T) stamp_row[(t * 4 + w) * 8 + (ev)] = (long long)__builtin_amdgcn_s_memtime();

  for (int t = 0; t < a.T; ++t) {
    LS_STAMP(0)

    floatx4 acc[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    if (t > 0) {
      // wait until the producers of h_{t-1}[my K range] have published step t-1
      const int p0 = w * nprod;
      unsigned spins = 0;
      while (!BC_ABL(a.dbg, 4)) {
        const unsigned f = lane < nprod ? __hip_atomic_load(flags + p0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                        : 0xffffffffu;
        if (__all(f >= (unsigned)t)) break;
        if (++spins > a.spin_limit) {
          if (lane == 0) {
            atomicAdd(a.status, 1);
            atomicAdd(a.status_total, 1);
            bail = 1;
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      // compiler ordering only (keeps the loads below the poll); visibility comes from the sc1 loads
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      LS_STAMP(1)
      // h_{t-1}: sc1 loads of slot t-1 (the hand-off form at the top of the file).
      // h arrives already split into its three bf16 planes (the producer splits once), as MFMA B
      // fragments: 3 x 16 B per lane per (k-step, n-tile).  Register double buffer: the 12 loads of
      // k-step ks+1 are in flight while k-step ks runs its 48 MFMAs (one wave per SIMD: nothing else
      // hides the L2 latency).
      const __amdgpu_buffer_rsrc_t hr = ls_rsrc(a.hseq + (long long)(t - 1) * hstep, (unsigned)(hstep * 4));
      ls_bf16x8 hbuf[2][4][3];
      auto load_ks = [&](int ks, ls_bf16x8 (&dst)[4][3]) {
        const int ksa = w * KS + ks;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int p = 0; p < 3; ++p)
            dst[nt][p] = ls_load_sc1<ls_bf16x8>(hr, (unsigned)((((ksa * 4 + nt) * 3 + p) * 64 + lane) * 16));
      };
      load_ks(0, hbuf[0]);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) load_ks(ks + 1, hbuf[(ks + 1) & 1]);
        // keep the scheduler from sinking those loads to their uses (it does under this register
        // pressure, serialising 144 L2 round trips per step)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const ls_bf16x8* hb = hbuf[ks & 1][nt];
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            floatx4 s = acc[mt][nt];
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][2], hb[0], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][1], hb[1], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][0], hb[2], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][1], hb[0], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][0], hb[1], s, 0, 0, 0);
            s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][0], hb[0], s, 0, 0, 0);
            acc[mt][nt] = s;
          }
        }
      }
    }

    // ---- reduce the four waves' partial sums (fixed order), cell update ----
    LS_STAMP(2)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) red[w][mt * 4 + nt][lane] = acc[mt][nt];
    __syncthreads();
    LS_STAMP(3)
    if (bail) return;  // uniform: every wave reads it after the same barrier
    float hq[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = 2 * w + q;
      floatx4 hsum = red[0][p][lane];
#pragma unroll
      for (int ww = 1; ww < LS_WAVES; ++ww) {
        const floatx4 r = red[ww][p][lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) hsum[i] = hsum[i] + r[i];
      }
      float gt[4];
#pragma unroll
      for (int gate = 0; gate < 4; ++gate) gt[gate] = t > 0 ? gxv[q][gate] + hsum[gate] : gxv[q][gate];
      const float ig = ls_sigmoid(gt[0]);
      const float fg = ls_sigmoid(gt[1]);
      const float gg = ls_tanh(gt[2]);
      const float og = ls_sigmoid(gt[3]);
      const float c = fg * cst[q] + ig * gg;
      cst[q] = c;
      hq[q] = cb[q] < a.nb ? og * ls_tanh(c) : 0.f;
      hs[cb[q]][cu[q]] = hq[q];
    }
    LS_STAMP(4)
    __syncthreads();
    LS_STAMP(5)

    // ---- publish h_t: wave 0, one clip per lane: split once into the three bf16 planes (the
    //      consumers' MFMA B fragments), 3 x 16 B write-through, drained, then the flag ----
    if (w == 0 && t + 1 < a.T) {
      const int b = lane, nt = b >> 4, c16 = b & 15;
      const int ksa = g >> 2, qq = g & 3;
      const __amdgpu_buffer_rsrc_t hr = ls_rsrc(a.hseq + (long long)t * hstep, (unsigned)(hstep * 4));
      const unsigned off = (unsigned)((ksa * 4 + nt) * 3 * 1024 + (qq * 16 + c16) * 16);
      float hv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) hv[i] = hs[b][i];
      ls_bf16x8 pl[3];
      ls_split8(hv, pl);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ls_u32x4, pl[p]), hr, off + p * 1024, 0, LS_SC1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(flags + g, (unsigned)(t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    LS_STAMP(6)
    // layer output (read only after the launch): off the publishing wave's critical path
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (cb[q] < a.nb) {
        const long long yi = (long long)(g * LS_U + cu[q]) * TB + (long long)t * a.Btot + a.b0 + cb[q];
        if (BC_DOK(yi < (long long)H * TB)) a.y[yi] = hq[q];
      }
    // next step's input-projection gates: issued after this step's publish drain so that drain does
    // not wait for them; they land during the next step's poll and MFMAs
    if (t + 1 < a.T) {
      load_gx(t + 1, gxn);
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int gate = 0; gate < 4; ++gate) gxv[q][gate] = gxn[q][gate];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Two interleaved half-batches (default).  The 64 clips of a launch are two independent
// recurrences of 32 clips; every workgroup alternates half 0 and half 1, so the hand-off of one
// half's h_t (write-through, flag, other workgroups' polls, fabric fetch: ~5 us, stamped timeline
// in DESIGN.md) overlaps the MFMAs of the other half instead of stalling the whole step.  The
// publishing wave also defers its flag store (and the drain before it) until after the next
// half-step's MFMAs, when the write-through stores have long completed.
//   hseq[t][half][k-step][n-tile (2)][plane][lane][8 bf16]; flags[half][G]; one cell per thread per
//   half (tile p = wave: m-tile p>>1, n-tile p&1).
// ------------------------------------------------------------------------------------------------
// P = 3: x6 (3 bf16 planes, 6 products).  P = 2: h3 (2 fp16 planes, 3 products, x6_common.h): W_hh
// rows are pre-scaled on the host by 2^(14 - e_row) (1 / scale stored after the planes), h_t in
// (-1, 1) is split with the fixed scale 2^14, and the summed gate products are unscaled per gate row.
// NTH: 16-clip n-tiles per half.  2 (halves of 32) for launches of 33-64 clips; 1 (halves of 16) for <= 32
// clips (BASELINE config 5 runs 32 per GPU), where halves of 32 left half 1 empty -- every step still paid its
// poll / load / reduction / publish chain for no clips.  Same hseq layout (n-tile 1 unused), same per-cell
// arithmetic in the same order: a clip's outputs do not depend on NTH (test_reslstm_half_split_bit_identical).
template <int KS, int P, int NTH = 2>
__global__ void __launch_bounds__(256, 1) lstm_seq2_x6_kernel(LstmSeqArgs a) {
  typedef typename LsFrag<P>::type frag_t;
  static_assert(NTH == 1 || NTH == 2, "halves of 16 or 32 clips");
  constexpr int NH = 16 * NTH;                 // clips per half
  __shared__ floatx4 red[LS_WAVES][4][64];     // per-wave partial gates of one half's 4 tiles
  __shared__ float hs[NH][LS_U + 1];           // one half's h_t gathered per clip
  __shared__ int bail;

  const int g = blockIdx.x;
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H;
  const long long TB = (long long)a.T * a.Btot;
  if (tid == 0) bail = 0;

  frag_t wr[2][KS][P];
  {
    const frag_t* wp = reinterpret_cast<const frag_t*>(a.whh) + (long long)(g * LS_WAVES + w) * (2 * KS * P) * 64 + lane;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int p = 0; p < P; ++p) wr[mt][ks][p] = wp[((mt * KS + ks) * P + p) * 64];
  }

  const int cu = (w >> 1) * 4 + (lane >> 4);   // my cell's unit within the workgroup
  // P == 2: 1 / (row scale * h scale 2^14) of my cell's four gate rows
  float gsc[4] = {1.f, 1.f, 1.f, 1.f};
  if constexpr (P == 2) {
    const float* wsc = reinterpret_cast<const float*>(a.whh + (long long)4 * H * H * P);
#pragma unroll
    for (int gate = 0; gate < 4; ++gate) gsc[gate] = wsc[gate * H + g * LS_U + cu] * (1.0f / 16384.0f);
  }
  const int cbh = (w & 1) * 16 + (lane & 15);  // my cell's clip within a half
  const bool cell = cbh < NH;                  // NTH == 1: waves 1 and 3 hold no cell
  float cst0 = 0.f, cst1 = 0.f;                // my cell's c in half 0 / half 1
  const long long unit_row = (long long)(g * LS_U + cu) * a.Btot + a.b0;  // [H][Btot] state row of my cell
  if (a.c0 && cell) {
    if (cbh < a.nb) cst0 = a.c0[unit_row + cbh];
    if (NH + cbh < a.nb) cst1 = a.c0[unit_row + NH + cbh];
  }

  const long long hhalf = (long long)H * (LS_NB * P / 2 / 2);  // floats of hseq per half-step
  const int nprod = G / LS_WAVES;
  const int sh = a.h0 ? 1 : 0;  // hseq slot shift: slot 0 = h0

  // h_t (or h0) of one half: gathered per clip in hs, split and written by wave 0 to hseq slot `slot`
  auto publish_slot = [&](int slot, int h) {
    if (w == 0 && lane < NH) {
      const int nt = lane >> 4, c16 = lane & 15;
      const int ksa = g >> 2, qq = g & 3;
      const __amdgpu_buffer_rsrc_t hr = ls_rsrc(a.hseq + ((long long)slot * 2 + h) * hhalf, (unsigned)(hhalf * 4));
      const unsigned off = (unsigned)((ksa * 2 + nt) * P * 1024 + (qq * 16 + c16) * 16);
      float hv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) hv[i] = hs[lane][i];
      ls_u32x4 pl[P];
      if constexpr (P == 2) {
        unsigned hh[4], mm[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) split2_h(hv[2 * i] * 16384.0f, hv[2 * i + 1] * 16384.0f, hh[i], mm[i]);
        pl[0] = (ls_u32x4){hh[0], hh[1], hh[2], hh[3]};
        pl[1] = (ls_u32x4){mm[0], mm[1], mm[2], mm[3]};
      } else {
        ls_bf16x8 pb[3];
        ls_split8(hv, pb);
#pragma unroll
        for (int p = 0; p < 3; ++p) pl[p] = __builtin_bit_cast(ls_u32x4, pb[p]);
      }
#pragma unroll
      for (int p = 0; p < P; ++p) __builtin_amdgcn_raw_buffer_store_b128(pl[p], hr, off + p * 1024, 0, LS_SC1);
    }
  };
  if (a.h0) {  // publish h0 of both halves to slot 0, then flags 1 (consumers of step 0 poll for them)
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      const int clip = h * NH + cbh;
      if (cell) hs[cbh][cu] = clip < a.nb ? a.h0[unit_row + clip] : 0.f;
      __syncthreads();
      publish_slot(0, h);
      __syncthreads();
    }
    if (w == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        __hip_atomic_store(a.flags + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.flags + 256 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  ls_gu32* flags = (ls_gu32*)(a.flags);
  int pend_h = -1;        // wave 0: half whose h stores are issued but whose flag is not yet set
  unsigned pend_v = 0;

  long long* stamp_row = nullptr;
  if (a.stamps && lane == 0 && (g == 0 || g == G / 2)) stamp_row = a.stamps + (long long)(g == 0 ? 0 : 1) * LS_STAMP_T * 32;

  for (int t = 0; t < a.T; ++t) {
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      const int ts = 2 * t + h;  // stamp row
#define LS2_STAMP(ev) \
  if (stamp_row && ts < LS_STAMP_T) stamp_row[(ts * 4 + w) * 8 + (ev)] = (long long)__builtin_amdgcn_s_memtime();
      LS2_STAMP(0)
      const int clip = h * NH + cbh;
      const bool ok = cell && clip < a.nb;
      float gxv[4];
#pragma unroll
      for (int gate = 0; gate < 4; ++gate)
        gxv[gate] = ok ? a.gx[((long long)gate * H + g * LS_U + cu) * TB + (long long)t * a.Btot + a.b0 + clip] : 0.f;

      floatx4 acc[2][2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

      if (t + sh > 0) {
        const ls_gu32* fl = flags + h * 256 + w * nprod;
        unsigned spins = 0;
        while (!BC_ABL(a.dbg, 4)) {
          const unsigned f = lane < nprod ? __hip_atomic_load(fl + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                          : 0xffffffffu;
          if (__all(f >= (unsigned)(t + sh))) break;
          if (++spins > a.spin_limit) {
            if (lane == 0) {
              atomicAdd(a.status, 1);
              atomicAdd(a.status_total, 1);
              bail = 1;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        // compiler ordering only (keeps the loads below the poll); visibility comes from the sc1 loads
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        LS2_STAMP(1)
        // h_{t-1} of this half: sc1 loads (the hand-off form at the top of the file)
        const __amdgpu_buffer_rsrc_t hr = ls_rsrc(a.hseq + ((long long)(t - 1 + sh) * 2 + h) * hhalf,
                                                  (unsigned)(hhalf * 4));
        // h_{t-1} fragments through a register ring LS_HD k-steps deep: the loads of k-step ks + LS_HD - 1
        // are issued before k-step ks's MFMAs, so L2 latency hides behind LS_HD - 1 k-steps of MFMAs
        // (depth 2 left ~2300 of a half-step's 4600 load+MFMA cycles exposed, profiles/r01g_lstm_h3_stamps.txt)
        constexpr int HD = LS_HD < KS ? LS_HD : KS;
        frag_t hbuf[HD][2][P];
        auto load_ks = [&](int ks, frag_t (&dst)[2][P]) {
          const int ksa = w * KS + ks;
#pragma unroll
          for (int nt = 0; nt < NTH; ++nt)
#pragma unroll
            for (int p = 0; p < P; ++p)
              dst[nt][p] = ls_load_sc1<frag_t>(hr, (unsigned)((((ksa * 2 + nt) * P + p) * 64 + lane) * 16));
        };
#pragma unroll
        for (int ks = 0; ks + 1 < HD; ++ks) load_ks(ks, hbuf[ks]);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          if (ks + HD - 1 < KS) load_ks(ks + HD - 1, hbuf[(ks + HD - 1) % HD]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int nt = 0; nt < NTH; ++nt) {
            const frag_t* hb = hbuf[ks % HD][nt];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
              floatx4 s = acc[mt][nt];
              if constexpr (P == 2) {
                s = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[mt][ks][1], hb[0], s, 0, 0, 0);
                s = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[mt][ks][0], hb[1], s, 0, 0, 0);
                s = __builtin_amdgcn_mfma_f32_16x16x32_f16(wr[mt][ks][0], hb[0], s, 0, 0, 0);
                acc[mt][nt] = s;
                continue;
              } else {
              s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][2], hb[0], s, 0, 0, 0);
              s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][1], hb[1], s, 0, 0, 0);
              s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][0], hb[2], s, 0, 0, 0);
              s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][1], hb[0], s, 0, 0, 0);
              s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][0], hb[1], s, 0, 0, 0);
              s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[mt][ks][0], hb[0], s, 0, 0, 0);
              acc[mt][nt] = s;
              }
            }
          }
        }
      }
      LS2_STAMP(2)
      // deferred flag of the previous half-step's publish: its stores were issued a whole
      // half-step ago, so this drain is (nearly) free
      if (w == 0 && pend_h >= 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(flags + pend_h * 256 + g, pend_v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pend_h = -1;
      }

#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) red[w][mt * 2 + nt][lane] = acc[mt][nt];
      __syncthreads();
      LS2_STAMP(3)
      if (bail) return;
      floatx4 hsum = red[0][w][lane];
#pragma unroll
      for (int ww = 1; ww < LS_WAVES; ++ww) {
        const floatx4 r = red[ww][w][lane];
#pragma unroll
        for (int i = 0; i < 4; ++i) hsum[i] = hsum[i] + r[i];
      }
      float gt[4];
#pragma unroll
      for (int gate = 0; gate < 4; ++gate)
        gt[gate] = t + sh > 0 ? gxv[gate] + (P == 2 ? hsum[gate] * gsc[gate] : hsum[gate]) : gxv[gate];
      const float ig = ls_sigmoid(gt[0]);
      const float fg = ls_sigmoid(gt[1]);
      const float gg = ls_tanh(gt[2]);
      const float og = ls_sigmoid(gt[3]);
      const float c = fg * (h ? cst1 : cst0) + ig * gg;
      if (h) cst1 = c;
      else cst0 = c;
      const float hq = ok ? og * ls_tanh(c) : 0.f;
      if (cell) hs[cbh][cu] = hq;
      LS2_STAMP(4)
      __syncthreads();
      LS2_STAMP(5)

      if (t + 1 < a.T) publish_slot(t + sh, h);
      if (w == 0 && t + 1 < a.T) {
        pend_h = h;
        pend_v = (unsigned)(t + 1 + sh);
      }
      LS2_STAMP(6)
      if (ok) {
        const long long yi = (long long)(g * LS_U + cu) * TB + (long long)t * a.Btot + a.b0 + clip;
        if (BC_DOK(yi < (long long)a.H * TB)) a.y[yi] = hq;
      }
      if (t + 1 == a.T && ok) {  // carried state out
        if (a.hT) a.hT[unit_row + clip] = hq;
        if (a.cT) a.cT[unit_row + clip] = c;
      }
#undef LS2_STAMP
    }
  }
  // no flag can still be pending: the last step publishes nothing
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
bool lstm_seq_ok(int H) {
  if (H % 128) return false;
  const int ks = H / 128;
  return ks == 2 || ks == 4 || ks == 8 || ks == 12;
}

// planes 3 (x6) or 2 (h3: + 1 / row scale per gate row, 4H floats)
long long lstm_seq_packed_bytes(int H, int planes) {
  return (long long)4 * H * H * planes * 2 + (planes == 2 ? (long long)4 * H * 4 : 0);
}

static inline unsigned short ls_f2bf(float f) {
  unsigned u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40);
  return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static inline float ls_bf2f(unsigned short h) {
  const unsigned u = (unsigned)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static inline unsigned short ls_f2h(float f) {
  const _Float16 h = (_Float16)f;
  unsigned short u;
  memcpy(&u, &h, 2);
  return u;
}
static inline float ls_h2f(unsigned short u) {
  _Float16 h;
  memcpy(&h, &u, 2);
  return (float)h;
}

// w: torch weight_hh [4H][H] (rows i, f, g, o).  out: [g][wave][mt][ks][plane][lane][8] bf16 (planes
// = 3) or fp16 of w * S_row (planes = 2, then 1 / S_row for the 4H rows in torch order)
void lstm_seq_pack(const float* w, unsigned short* out, int H, int planes) {
  const int KS = H / 128, G = H / LS_U;
  std::vector<float> rsc(planes == 2 ? (size_t)4 * H : 0, 1.f);
  for (size_t row = 0; row < rsc.size(); ++row) {
    float m = 0.f;
    for (int k = 0; k < H; ++k) m = std::max(m, std::fabs(w[(long long)row * H + k]));
    if (m > 0.f && std::isfinite(m)) rsc[row] = std::ldexp(1.f, 14 - std::max(-112, std::min(140, std::ilogb(m))));
  }
  long long o = 0;
  for (int g = 0; g < G; ++g)
    for (int wv = 0; wv < LS_WAVES; ++wv)
      for (int mt = 0; mt < 2; ++mt)
        for (int ks = 0; ks < KS; ++ks)
          for (int p = 0; p < planes; ++p)
            for (int lane = 0; lane < 64; ++lane)
              for (int j = 0; j < 8; ++j, ++o) {
                const int m = lane & 15;
                const int unit = g * LS_U + mt * 4 + (m >> 2);
                const int row = (m & 3) * H + unit;
                const int k = (wv * KS + ks) * 32 + 8 * (lane >> 4) + j;
                const float v = w[(long long)row * H + k];
                if (planes == 2) {
                  const float vs = v * rsc[row];
                  const unsigned short g0 = ls_f2h(vs);
                  out[o] = p == 0 ? g0 : ls_f2h(vs - ls_h2f(g0));
                  continue;
                }
                const unsigned short h0 = ls_f2bf(v);
                const float r1 = v - ls_bf2f(h0);
                const unsigned short h1 = ls_f2bf(r1);
                const unsigned short h2 = ls_f2bf(r1 - ls_bf2f(h1));
                out[o] = p == 0 ? h0 : p == 1 ? h1 : h2;
              }
  if (planes == 2) {
    float* inv = reinterpret_cast<float*>(out + o);
    for (size_t row = 0; row < rsc.size(); ++row) inv[row] = 1.f / rsc[row];
  }
}

long long lstm_seq_workspace_bytes(int H, int T) {
  return LS_FLAG_BYTES + (long long)(T + 1) * H * LS_HSTEP_PER_UNIT * 4;  // flags [2][256] | hseq (+ h0 slot)
}

__device__ int bc_lstm_seq_timeouts;  // bumped by a workgroup that gave up waiting (never in a good run)

static int* status_word() {
  static int* p = [] {
    void* q = nullptr;
    if (hipGetSymbolAddress(&q, HIP_SYMBOL(bc_lstm_seq_timeouts)) != hipSuccess) return (int*)nullptr;
    return reinterpret_cast<int*>(q);
  }();
  return p;
}

int lstm_seq_read_status(int reset) {
  int v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(bc_lstm_seq_timeouts), sizeof(int)) != hipSuccess) return -1;
  if (reset) {
    const int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(bc_lstm_seq_timeouts), &z, sizeof(int)) != hipSuccess) return -1;
  }
  return v;
}

// Diagnostic stamp buffer (BC_LSTM_SEQ_STAMPS=1): allocated once, read by bc_debug_lstm_stamps.
static long long* lstm_seq_stamp_buffer() {
  static long long* p = [] {
    const char* e = getenv("BC_LSTM_SEQ_STAMPS");
    long long* q = nullptr;
    if (e && atoi(e) && hipMalloc(&q, sizeof(long long) * 2 * LS_STAMP_T * 32) != hipSuccess) q = nullptr;
    return q;
  }();
  return p;
}

static unsigned g_spin_limit = LS_SPIN_LIMIT;

static int device_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return v;
  }();
  return n;
}

// Every workgroup of a persistent launch must be resident at once (they wait on each other's flags):
// G <= CUs x the kernel's occupancy per CU at 256 threads (its registers / LDS), checked per kernel.
template <typename K>
static bool all_resident(K kernel, int G) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess) return false;
  return per_cu >= 1 && (long long)G <= (long long)per_cu * device_cus();
}

static bool seq_resident(int KS, int planes, bool halves, int G) {
#define BC_LS_RES(K)                                                                        \
  case K:                                                                                   \
    if (planes == 2)                                                                        \
      return all_resident(lstm_seq2_x6_kernel<K, 2>, G) && all_resident(lstm_seq2_x6_kernel<K, 2, 1>, G); \
    if (halves) return all_resident(lstm_seq2_x6_kernel<K, 3>, G) && all_resident(lstm_seq2_x6_kernel<K, 3, 1>, G); \
    return all_resident(lstm_seq_x6_kernel<K>, G);
  switch (KS) {
    BC_LS_RES(2)
    BC_LS_RES(4)
    BC_LS_RES(8)
    BC_LS_RES(12)
    default: return false;
  }
#undef BC_LS_RES
}

int lstm_seq_launch(const float* gx, const unsigned short* whh, float* y, void* ws, int H, int T, int Btot,
                    int planes, hipStream_t st, const float* h0, const float* c0, float* hT, float* cT,
                    int* call_status) {
  if (planes != 2 && planes != 3) return BC_ERR_ARG;
  if (!lstm_seq_ok(H)) return BC_ERR_UNSUPPORTED;
  const int G = H / LS_U;
  if (G > 256 || G > device_cus()) return BC_ERR_UNSUPPORTED;  // every workgroup must be resident
  int* status = status_word();
  if (!status) return BC_ERR_LAUNCH;
  LstmSeqArgs a{};
  a.gx = gx;
  a.whh = whh;
  a.y = y;
  a.flags = reinterpret_cast<unsigned*>(ws);
  a.hseq = reinterpret_cast<float*>(reinterpret_cast<unsigned char*>(ws) + LS_FLAG_BYTES);
  a.status = call_status ? call_status : status;
  a.status_total = status;
  a.spin_limit = g_spin_limit;
  a.H = H;
  a.T = T;
  a.Btot = Btot;
  static const int dbg = [] {
    const char* e = getenv("BC_LSTM_SEQ_DEBUG");
    return e ? atoi(e) : 0;
  }();
  a.dbg = dbg;
  a.stamps = lstm_seq_stamp_buffer();
  a.h0 = h0;
  a.c0 = c0;
  a.hT = hT;
  a.cT = cT;
  // BC_LSTM_SEQ_HALVES=1: the single-batch kernel (kept for A/B timing), else two interleaved halves
  static const bool halves = [] {
    const char* e = getenv("BC_LSTM_SEQ_HALVES");
    return !(e && atoi(e) == 1);
  }();
  if (!halves && (h0 || c0 || hT || cT)) return BC_ERR_UNSUPPORTED;  // carried state: lstm_seq2 only
  static int resident_checked[4][2] = {};  // per (H/128 case, kernel): 1 ok, -1 refused
  const int ks_idx = H == 256 ? 0 : H == 512 ? 1 : H == 1024 ? 2 : 3;
  int& rs = resident_checked[ks_idx][planes == 2 ? 0 : 1];
  if (rs == 0) rs = seq_resident(H / 128, planes, halves, G) ? 1 : -1;
  if (rs < 0) return BC_ERR_UNSUPPORTED;
  // BC_LSTM_NH16=0 keeps launches of <= 32 clips on halves of 32 (A/B timing)
  static const bool nh16 = [] {
    const char* e = getenv("BC_LSTM_NH16");
    return !(e && atoi(e) == 0);
  }();
  for (int b0 = 0; b0 < Btot; b0 += LS_NB) {
    a.b0 = b0;
    a.nb = Btot - b0 < LS_NB ? Btot - b0 : LS_NB;
    const bool h16 = nh16 && a.nb <= 32;
    if (hipMemsetAsync(a.flags, 0, LS_FLAG_BYTES, st) != hipSuccess) return BC_ERR_LAUNCH;
#define BC_LS_CASE(KS)                                                                      \
  case KS:                                                                                  \
    if (planes == 2 && h16)                                                                 \
      hipLaunchKernelGGL((lstm_seq2_x6_kernel<KS, 2, 1>), dim3(G), dim3(256), 0, st, a);    \
    else if (planes == 2)                                                                   \
      hipLaunchKernelGGL((lstm_seq2_x6_kernel<KS, 2>), dim3(G), dim3(256), 0, st, a);       \
    else if (halves && h16)                                                                 \
      hipLaunchKernelGGL((lstm_seq2_x6_kernel<KS, 3, 1>), dim3(G), dim3(256), 0, st, a);    \
    else if (halves)                                                                        \
      hipLaunchKernelGGL((lstm_seq2_x6_kernel<KS, 3>), dim3(G), dim3(256), 0, st, a);       \
    else                                                                                    \
      hipLaunchKernelGGL(lstm_seq_x6_kernel<KS>, dim3(G), dim3(256), 0, st, a);             \
    break;
    switch (H / 128) {
      BC_LS_CASE(2)
      BC_LS_CASE(4)
      BC_LS_CASE(8)
      BC_LS_CASE(12)
      default: return BC_ERR_UNSUPPORTED;
    }
#undef BC_LS_CASE
    BC_CHECK_LAUNCH();
  }
  return BC_OK;
}

// the symbol of the launch lstm_seq_launch makes for a launch of nb clips (its dispatch above; the launch timer)
const char* lstm_seq_kernel_name(int H, int planes, int nb) {
  static thread_local char buf[64];
  const char* e = getenv("BC_LSTM_SEQ_HALVES");
  const bool halves = !(e && atoi(e) == 1);
  const char* e16 = getenv("BC_LSTM_NH16");
  const bool h16 = !(e16 && atoi(e16) == 0) && nb <= 32;
  const int ks = H / 128;
  if (planes != 2 && !halves)
    snprintf(buf, sizeof buf, "lstm_seq_x6_kernel<%d>", ks);
  else
    snprintf(buf, sizeof buf, "lstm_seq2_x6_kernel<%d, %d, %d>", ks, planes, h16 ? 1 : 2);  // (NTH spelled out, as
                                                                                               // rocprofv3 names it)
  return buf;
}

}  // namespace bc

// Diagnostics only (not part of include/bigcodec.h): override the persistent kernel's poll limit
// (limit 0 = restore the default).  Tests force the timeout path with a tiny limit.
extern "C" int bc_debug_set_lstm_spin_limit(long long limit) {
  if (limit < 0 || limit > 0xffffffffLL) return 1;
  bc::g_spin_limit = limit == 0 ? bc::LS_SPIN_LIMIT : (unsigned)limit;
  return 0;
}

// Diagnostics only (not part of include/bigcodec.h): copy the last persistent launch's stamps
// [2 workgroups][2048 steps][4 waves][8 events] (s_memtime ticks) to the host; synchronises.
extern "C" int bc_debug_lstm_stamps(long long* host, long long n) {
  long long* p = bc::lstm_seq_stamp_buffer();
  if (!p || !host || n <= 0 || n > 2LL * bc::LS_STAMP_T * 32) return 1;
  return hipMemcpy(host, p, sizeof(long long) * n, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}

BC_DEBUG_EXPORT(lstm_seq)
