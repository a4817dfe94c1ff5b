// extern "C" entry points of libbigcodec_hip.so (declared and documented in include/bigcodec.h).
#include "../../include/bigcodec.h"
#include "bc_common.h"
#include "bc_internal.h"

#include <cstdio>
#include <mutex>
#include <string>
#include <vector>

using namespace bc;

// ---- launch timer (bc_launch_timer_*): HIP events around the launches of the composite calls ----
namespace bc {
namespace {
struct LTRec {
  std::string name;
  hipEvent_t e0, e1;
  double flops, bytes;
};
std::mutex g_lt_mu;
bool g_lt_on = false;
std::vector<LTRec> g_lt;
std::vector<hipEvent_t> g_lt_pool;
hipEvent_t lt_event() {
  if (!g_lt_pool.empty()) {
    hipEvent_t e = g_lt_pool.back();
    g_lt_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
}  // namespace

LTScope::LTScope(const char* name, double flops, double bytes, hipStream_t st) : idx(-1) {
  std::lock_guard<std::mutex> lk(g_lt_mu);
  if (!g_lt_on) return;
  hipEvent_t e0 = lt_event(), e1 = lt_event();
  if (!e0 || !e1 || hipEventRecord(e0, st) != hipSuccess) return;
  g_lt.push_back({name, e0, e1, flops, bytes});
  idx = (int)g_lt.size() - 1;
  st_ = st;
}
LTScope::~LTScope() {
  if (idx < 0) return;
  std::lock_guard<std::mutex> lk(g_lt_mu);
  if (idx < (int)g_lt.size()) (void)hipEventRecord(g_lt[idx].e1, st_);
}
}  // namespace bc


static inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

extern "C" {

static void lt_clear() {  // (caller holds g_lt_mu)
  for (auto& r : bc::g_lt) {
    bc::g_lt_pool.push_back(r.e0);
    bc::g_lt_pool.push_back(r.e1);
  }
  bc::g_lt.clear();
}

int bc_launch_timer_enable(int on) {
  std::lock_guard<std::mutex> lk(bc::g_lt_mu);
  if (on && !bc::g_lt_on) lt_clear();  // a fresh recording
  bc::g_lt_on = on != 0;
  return BC_OK;
}

int bc_launch_timer_read(int max, char* names, float* ms, double* flops, double* bytes) {
  std::lock_guard<std::mutex> lk(bc::g_lt_mu);
  const int n = (int)bc::g_lt.size();
  if (!names || !ms || !flops || !bytes || max <= 0) return n;  // the count only; nothing is cleared
  int rc = n;
  for (int i = 0; i < n; ++i) {
    auto& r = bc::g_lt[i];
    if (i < max) {
      float t = 0.f;
      if (hipEventSynchronize(r.e1) != hipSuccess || hipEventElapsedTime(&t, r.e0, r.e1) != hipSuccess) rc = -1;
      snprintf(names + 64 * (long long)i, 64, "%s", r.name.c_str());
      ms[i] = t;
      flops[i] = r.flops;
      bytes[i] = r.bytes;
    }
  }
  lt_clear();
  return rc;
}


int bc_abi_version(void) { return BC_ABI_VERSION; }

int bc_conv1d_select_cfg(int Cout, int Cin, int K, int stride, int dilation, int mode) {
  if (Cout <= 0 || Cin <= 0 || K <= 0 || stride <= 0 || dilation <= 0) return -1;
  if (mode < 0 || mode > 3) return -1;
  return conv_select_cfg(Cout, Cin, K, stride, dilation, mode);
}

static int device_cus() {
  static const int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return cus;
}

int bc_conv1d_select_cfg_n(int Cout, int Cin, int K, int stride, int dilation, int mode, int B, int Tout) {
  const int cfg = bc_conv1d_select_cfg(Cout, Cin, K, stride, dilation, mode);
  if (cfg < 0 || mode < 1) return cfg;
  return x6_narrow_cfg(cfg, Cout, K, stride, dilation, mode == 1 ? 3 : mode == 2 ? 1 : 2, B, Tout, device_cus());
}

// a cfg is acceptable for a shape if some precision mode selects it
// Any valid tile id may run a conv (the select functions give the tuned choice; tools/conv_bench.py
// times others): the kernel launchers reject a tile the shape does not fit (BC_ERR_UNSUPPORTED).
// A phase-decomposed id (1000 * s + tile) only runs stride-s, dilation-1 convs.
static bool cfg_matches(int cfg, int Cout, int Cin, int K, int s, int d) {
  (void)Cout; (void)Cin; (void)K;
  if (cfg >= 1000) return cfg / 1000 == s && d == 1;
  return true;
}

long long bc_conv1d_packed_floats(int Cout, int Cin, int K, int cfg) {
  if (Cout <= 0 || Cin <= 0 || K <= 0 || !conv_cfg_valid(cfg)) return -1;
  return conv_packed_floats(Cout, Cin, K, cfg);
}

int bc_conv1d_pack(const float* w_host, float* packed_host, int Cout, int Cin, int K, int cfg) {
  if (!w_host || !packed_host || Cout <= 0 || Cin <= 0 || K <= 0 || !conv_cfg_valid(cfg))
    return BC_ERR_ARG;
  conv_pack_weight(w_host, packed_host, Cout, Cin, K, cfg);
  return BC_OK;
}

int bc_conv1d_fwd(const float* x, const float* w_packed, const float* bias, const float* residual,
                  const float* out_snake_alpha_exp, const float* out_snake_inv_beta, float* y,
                  float* y2, int B, int Cin, int Tin, int Cout, int Tout, int K, int stride,
                  int dilation, int pad_left, int epilogue, int cfg, void* stream) {
  if (!x || !w_packed || !y || B < 0 || Cin <= 0 || Tin < 0 || Cout <= 0 || Tout < 0 || K <= 0 ||
      stride <= 0 || dilation <= 0 || pad_left < 0 || !conv_cfg_valid(cfg))
    return BC_ERR_ARG;
  if ((out_snake_alpha_exp == nullptr) != (out_snake_inv_beta == nullptr)) return BC_ERR_ARG;
  if (y2 && !out_snake_alpha_exp) return BC_ERR_ARG;
  if (epilogue != 0 && epilogue != 1) return BC_ERR_ARG;
  if (epilogue == 1 && out_snake_alpha_exp) return BC_ERR_ARG;
  if (!cfg_matches(cfg, Cout, Cin, K, stride, dilation)) return BC_ERR_ARG;
  if (B == 0 || Tout == 0) return BC_OK;
  ConvArgs a{};
  a.x = x; a.w = w_packed; a.bias = bias; a.res = residual;
  a.osa = out_snake_alpha_exp; a.osb = out_snake_inv_beta; a.y = y; a.y2 = y2;
  a.xbs = (long long)Cin * Tin; a.ybs = (long long)Cout * Tout; a.rbs = a.ybs;
  a.Cin = Cin; a.Tin = Tin; a.Cout = Cout; a.Nout = Tout;
  a.K = K; a.s = stride; a.d = dilation; a.pl = pad_left;
  a.yT = Tout; a.ostride = 1; a.ooff = 0; a.epi = epilogue;
#ifdef BC_ABLATION
  // BC_ABL_PW_RAW_ONLY=1 (ablation builds, wrong results, timing): dual-output pointwise convs write the raw output only
  static const bool raw_only = getenv("BC_ABL_PW_RAW_ONLY") != nullptr;
  if (raw_only && K == 1 && y2) a.y2 = nullptr, a.osa = nullptr, a.osb = nullptr;
#endif
  return conv_launch(a, B, cfg, S(stream));
}

int bc_resunit_select_cfg(int C, int dilation, int mode) {
  if (C <= 0 || dilation <= 0) return -1;
  return resunit_select_cfg(C, dilation, mode);
}

int bc_resunit_fwd(const float* x_raw, const float* x_act, const float* w7_packed, const float* b7,
                   const float* mid_snake_alpha_exp, const float* mid_snake_inv_beta,
                   const float* w1_packed, const float* b1, const float* out_snake_alpha_exp,
                   const float* out_snake_inv_beta, float* y, float* y2, int B, int C, int T,
                   int dilation, int pad_left, int cfg, void* stream) {
  if (!x_raw || !x_act || !w7_packed || !w1_packed || !mid_snake_alpha_exp || !mid_snake_inv_beta || !y ||
      B < 0 || C <= 0 || T < 0 || dilation <= 0 || pad_left < 0 || pad_left > 6 * dilation)
    return BC_ERR_ARG;
  if ((out_snake_alpha_exp == nullptr) != (out_snake_inv_beta == nullptr)) return BC_ERR_ARG;
  if (y2 && !out_snake_alpha_exp) return BC_ERR_ARG;
  if (!resunit_cfg_ok(cfg, C, dilation)) return BC_ERR_ARG;
  if (B == 0 || T == 0) return BC_OK;
  return resunit_launch(x_raw, x_act, w7_packed, b7, mid_snake_alpha_exp, mid_snake_inv_beta, w1_packed, b1,
                        out_snake_alpha_exp, out_snake_inv_beta, y, y2, B, C, T, dilation, pad_left, cfg,
                        S(stream));
}

int bc_resunit_fwd_snake_in(const float* x_raw, const float* in_snake_alpha_exp, const float* in_snake_inv_beta,
                            const float* w7_packed, const float* b7, const float* mid_snake_alpha_exp,
                            const float* mid_snake_inv_beta, const float* w1_packed, const float* b1,
                            const float* out_snake_alpha_exp, const float* out_snake_inv_beta, float* y, float* y2,
                            int B, int C, int T, int dilation, int pad_left, int cfg, void* stream) {
  if (!x_raw || !in_snake_alpha_exp || !in_snake_inv_beta || !w7_packed || !w1_packed || !mid_snake_alpha_exp ||
      !mid_snake_inv_beta || !y || B < 0 || C <= 0 || T < 0 || dilation <= 0 || pad_left < 0 ||
      pad_left > 6 * dilation)
    return BC_ERR_ARG;
  if ((out_snake_alpha_exp == nullptr) != (out_snake_inv_beta == nullptr)) return BC_ERR_ARG;
  if (y2 && !out_snake_alpha_exp) return BC_ERR_ARG;
  if (!resunit_cfg_ok(cfg, C, dilation)) return BC_ERR_ARG;
  if (B == 0 || T == 0) return BC_OK;
  return resunit_launch(x_raw, x_raw, w7_packed, b7, mid_snake_alpha_exp, mid_snake_inv_beta, w1_packed, b1,
                        out_snake_alpha_exp, out_snake_inv_beta, y, y2, B, C, T, dilation, pad_left, cfg,
                        S(stream), in_snake_alpha_exp, in_snake_inv_beta);
}

int bc_convT1d_phase_taps(int K, int stride) {
  if (K <= 0 || stride <= 0) return -1;
  return (K + stride - 1) / stride;
}

// phase r of a transposed conv: outputs t = s*q - p + r for q in [q_lo, q_lo + nout)
static void convT_phase(int r, int s, int p, int Tout, int* q_lo, int* nout) {
  const int lo = (p - r + s - 1 >= 0) ? (p - r + s - 1) / s : -((r - p) / s);
  const long long q_hi_num = (long long)Tout - 1 + p - r;
  const int hi = q_hi_num >= 0 ? (int)(q_hi_num / s) : -1;
  *q_lo = lo;
  *nout = hi - lo + 1;
}
// contiguous per-phase rows of the workspace: Q4 = max phase length rounded up to 4 (16-byte epilogue rows)
static int convT_q4(int Tout, int s, int p) {
  int qmax = 0;
  for (int r = 0; r < s; ++r) {
    int lo, n;
    convT_phase(r, s, p, Tout, &lo, &n);
    qmax = n > qmax ? n : qmax;
  }
  return (qmax + 3) / 4 * 4;
}

long long bc_convT1d_workspace_floats(int B, int Cout, int Tout, int K, int stride, int padding, int dual) {
  if (B < 0 || Cout <= 0 || Tout < 0 || K <= 0 || stride <= 0 || stride > CONVT_MAX_STRIDE || padding < 0) return -1;
  return (long long)stride * B * Cout * convT_q4(Tout, stride, padding) * (dual ? 2 : 1);
}

int bc_convT1d_fwd_ws(const float* x, const float* const* w_phases, const float* bias,
                      const float* out_snake_alpha_exp, const float* out_snake_inv_beta, float* y,
                      float* y2, int B, int Cin, int Tin, int Cout, int Tout, int K, int stride,
                      int padding, int cfg, float* workspace, void* stream) {
  // BC_CONVT_DIRECT_MAXS=s: strides <= s take the strided-store path even with a workspace (A/B timing)
  static const int direct_maxs = [] {
    const char* e = getenv("BC_CONVT_DIRECT_MAXS");
    return e ? atoi(e) : 0;
  }();
  if (!workspace || stride <= direct_maxs)
    return bc_convT1d_fwd(x, w_phases, bias, out_snake_alpha_exp, out_snake_inv_beta, y, y2, B, Cin, Tin, Cout, Tout, K,
                          stride, padding, cfg, stream);
  if (!x || !w_phases || !y || B < 0 || Cin <= 0 || Tin < 0 || Cout <= 0 || Tout < 0 || K <= 0 || stride <= 0 ||
      stride > CONVT_MAX_STRIDE || padding < 0 || !conv_cfg_valid(cfg))
    return BC_ERR_ARG;
  if ((out_snake_alpha_exp == nullptr) != (out_snake_inv_beta == nullptr)) return BC_ERR_ARG;
  if (y2 && !out_snake_alpha_exp) return BC_ERR_ARG;
  const int s = stride, p = padding;
  const int Kp = (K + s - 1) / s;
  if (!cfg_matches(cfg, Cout, Cin, Kp, 1, 1)) return BC_ERR_ARG;
  if (B == 0 || Tout == 0) return BC_OK;
  const int Q4 = convT_q4(Tout, s, p);
  const long long plane = (long long)B * Cout * Q4;  // one phase's rows
  float* w2 = y2 ? workspace + s * plane : nullptr;
  ConvTInterleave il{};
  il.s = s;
  il.p = p;
  for (int r = 0; r < s; ++r) {
    if (!w_phases[r]) return BC_ERR_ARG;
    int q_lo, nout;
    convT_phase(r, s, p, Tout, &q_lo, &nout);
    il.q_lo[r] = q_lo;
    if (nout <= 0) continue;
    ConvArgs a{};
    a.x = x; a.w = w_phases[r]; a.bias = bias; a.res = nullptr;
    a.osa = out_snake_alpha_exp; a.osb = out_snake_inv_beta; a.y = workspace + r * plane; a.y2 = w2 ? w2 + r * plane : nullptr;
    a.xbs = (long long)Cin * Tin; a.ybs = (long long)Cout * Q4; a.rbs = 0;
    a.Cin = Cin; a.Tin = Tin; a.Cout = Cout; a.Nout = nout;
    a.K = Kp; a.s = 1; a.d = 1; a.pl = Kp - 1 - q_lo;  // as bc_convT1d_fwd
    a.yT = Q4; a.ostride = 1; a.ooff = 0; a.epi = 0;
    if (a.pl < 0) return BC_ERR_UNSUPPORTED;
    const int rc = conv_launch(a, B, cfg, S(stream));
    if (rc != BC_OK) return rc;
  }
  return convT_interleave_launch(workspace, w2, y, y2, B, Cout, Tout, Q4, il, S(stream));
}

int bc_convT1d_fwd(const float* x, const float* const* w_phases, const float* bias,
                   const float* out_snake_alpha_exp, const float* out_snake_inv_beta, float* y,
                   float* y2, int B, int Cin, int Tin, int Cout, int Tout, int K, int stride,
                   int padding, int cfg, void* stream) {
  if (!x || !w_phases || !y || B < 0 || Cin <= 0 || Tin < 0 || Cout <= 0 || Tout < 0 || K <= 0 ||
      stride <= 0 || padding < 0 || !conv_cfg_valid(cfg))
    return BC_ERR_ARG;
  if ((out_snake_alpha_exp == nullptr) != (out_snake_inv_beta == nullptr)) return BC_ERR_ARG;
  if (y2 && !out_snake_alpha_exp) return BC_ERR_ARG;
  const int s = stride, p = padding;
  const int Kp = (K + s - 1) / s;  // taps per phase
  if (!cfg_matches(cfg, Cout, Cin, Kp, 1, 1)) return BC_ERR_ARG;
  if (B == 0 || Tout == 0) return BC_OK;
  for (int r = 0; r < s; ++r) {
    if (!w_phases[r]) return BC_ERR_ARG;
    // outputs t = s*q - p + r, q in [q_lo, q_hi]
    const int q_lo = (p - r + s - 1 >= 0) ? (p - r + s - 1) / s : -((r - p) / s);
    const long long q_hi_num = (long long)Tout - 1 + p - r;
    const int q_hi = q_hi_num >= 0 ? (int)(q_hi_num / s) : -1;
    const int nout = q_hi - q_lo + 1;
    if (nout <= 0) continue;
    ConvArgs a{};
    a.x = x; a.w = w_phases[r]; a.bias = bias; a.res = nullptr;
    a.osa = out_snake_alpha_exp; a.osb = out_snake_inv_beta; a.y = y; a.y2 = y2;
    a.xbs = (long long)Cin * Tin; a.ybs = (long long)Cout * Tout; a.rbs = 0;
    a.Cin = Cin; a.Tin = Tin; a.Cout = Cout; a.Nout = nout;
    // Kp-tap conv: tap j' reads input q - (Kp-1) + j' (weight W[ci][co][r + s*(Kp-1-j')]);
    // q = n + q_lo
    a.K = Kp; a.s = 1; a.d = 1; a.pl = Kp - 1 - q_lo;
    a.yT = Tout; a.ostride = s; a.ooff = s * q_lo - p + r; a.epi = 0;
    if (a.pl < 0) return BC_ERR_UNSUPPORTED;  // padding >= K: not a DecoderBlock shape
    const int rc = conv_launch(a, B, cfg, S(stream));
    if (rc != BC_OK) return rc;
  }
  return BC_OK;
}

int bc_snake_fwd(const float* x, const float* snake_alpha_exp, const float* snake_inv_beta,
                 float* y, int B, int C, long long T, void* stream) {
  if (!x || !y || !snake_alpha_exp || !snake_inv_beta || B < 0 || C <= 0 || T < 0) return BC_ERR_ARG;
  return snake_launch(x, snake_alpha_exp, snake_inv_beta, y, B, C, T, S(stream));
}

long long bc_aa_snake_out_len(int T, int up_ratio, int down_ratio, int down_taps) {
  if (T < 0 || up_ratio < 1 || down_ratio < 1 || down_taps < 1) return -1;
  return aa_snake_out_len(T, up_ratio, down_ratio, down_taps);
}

int bc_aa_snake_fwd_ex(const float* x, const float* snake_alpha_exp, const float* snake_inv_beta,
                       const float* up_filter, const float* down_filter, float* y, int B, int C, int T, int up_ratio,
                       int up_taps, int down_ratio, int down_taps, void* stream) {
  if (!x || !y || !snake_alpha_exp || !snake_inv_beta || !up_filter || !down_filter || B < 0 || C <= 0 || T < 0 ||
      up_ratio < 1 || down_ratio < 1 || up_taps < 1 || down_taps < 1)
    return BC_ERR_ARG;
  if (up_ratio == 2 && down_ratio == 2 && up_taps == 12 && down_taps == 12)  // the reference's default: fixed kernel
    return aa_snake_launch(x, snake_alpha_exp, snake_inv_beta, up_filter, down_filter, y, B, C, T, S(stream));
  return aa_snake_gen_launch(x, snake_alpha_exp, snake_inv_beta, up_filter, down_filter, y, B, C, T, up_ratio, up_taps,
                             down_ratio, down_taps, S(stream));
}

int bc_aa_snake_fwd(const float* x, const float* snake_alpha_exp, const float* snake_inv_beta,
                    const float* up_filter, const float* down_filter, float* y, int B, int C, int T,
                    void* stream) {
  if (!x || !y || !snake_alpha_exp || !snake_inv_beta || !up_filter || !down_filter || B < 0 ||
      C <= 0 || T < 0)
    return BC_ERR_ARG;
  return aa_snake_launch(x, snake_alpha_exp, snake_inv_beta, up_filter, down_filter, y, B, C, T,
                         S(stream));
}

// The recurrence is accuracy-critical: mode 2 (bf16 conv products) keeps the LSTM fp32-class, on the h3
// arithmetic since round 3 (x6 before: the same accuracy class at ~2.8x the recurrence time).
// Mode 3 (h3) runs the input projection as an h3 conv and the recurrence as the h3 persistent kernel.
static int lstm_mode(int mode) { return mode == 2 ? 3 : mode; }
static bool lstm_use_seq(int H, int mode) {
  const int m = lstm_mode(mode);
  return (m == 1 || m == 3) && lstm_seq_ok(H);
}
static int lstm_planes(int mode) { return lstm_mode(mode) == 3 ? 2 : 3; }

long long bc_lstm_hh_packed_floats(int H, int mode) {
  if (H <= 0 || H % 16 || mode < 0 || mode > 3) return -1;
  if (lstm_use_seq(H, mode)) return lstm_seq_packed_bytes(H, lstm_planes(mode)) / 4;
  return (long long)4 * H * H;
}

int bc_lstm_status(int reset) { return lstm_seq_read_status(reset); }

int bc_mfma_probe(float* out, int nwg, int iters, void* stream) { return mfma_probe_launch(out, nwg, iters, S(stream)); }

int bc_lstm_pack_hh(const float* w_hh_host, float* packed_host, int H, int mode) {
  if (!w_hh_host || !packed_host || H <= 0 || H % 16 || mode < 0 || mode > 3) return BC_ERR_ARG;
  if (lstm_use_seq(H, mode))
    lstm_seq_pack(w_hh_host, reinterpret_cast<unsigned short*>(packed_host), H, lstm_planes(mode));  // persistent kernel
  else if (lstm_fast_ok(H))
    lstm_pack_hh2(w_hh_host, packed_host, H);  // layout of the register-resident fast step kernel
  else
    lstm_pack_hh(w_hh_host, packed_host, H);
  return BC_OK;
}

// workspace: status [64 floats: int32 timeout count of this call] | xt [H][T*B] | gx [4H][T*B] |
// y0 [H][T*B] | y1 [H][T*B] | c [H][B] | hfrag x2 or the persistent kernel's region | the input projection's
// pre-split B planes (pw_presplit.hip, h3 and x6)
constexpr long long LSTM_WS_STATUS_FLOATS = 64;
static long long lstm_frag_floats(int B, int H) { return (long long)((B + 63) / 64) * 64 * H; }
static long long lstm_ws_head_floats(int B, int H, int T) {
  const long long tb = (long long)T * B;
  const long long frag = 2 * lstm_frag_floats(B, H);
  const long long seq = lstm_seq_ok(H) ? lstm_seq_workspace_bytes(H, T) / 4 : 0;
  return (LSTM_WS_STATUS_FLOATS + tb * H * 3 + tb * 4 * H + (long long)H * B + (frag > seq ? frag : seq) + 3) / 4 * 4;
}
// The input projection on the pre-split GEMM (h3 and x6, Cout % 192 == 0, Cin % 32 == 0): on by default; BC_LSTM_PRESPLIT=0
// or bc_debug_set_lstm_presplit(0) runs it on conv1d_x6_kernel (A/B timing, the bit-identity test).
static int g_lstm_presplit = [] {
  const char* e = getenv("BC_LSTM_PRESPLIT");
  return e && atoi(e) == 0 ? 0 : 1;
}();

long long bc_lstm_workspace_floats(int B, int H, int T) {
  if (B < 0 || H <= 0 || T < 0) return -1;
  const long long tb = (long long)T * B;
  return lstm_ws_head_floats(B, H, T) + (pw_presplit_bytes(H, tb > 0 ? tb : 1) + 3) / 4;
}

static int reslstm_impl(const float* x, float* out, int B, int H, int T, int num_layers,
                        const float* const* w_ih_packed, const float* const* bias,
                        const float* const* w_hh_packed, const float* out_snake_alpha_exp,
                        const float* out_snake_inv_beta, float* workspace, int mode, void* stream,
                        const float* h0, const float* c0, float* hT, float* cT);

int bc_reslstm_fwd(const float* x, float* out, int B, int H, int T, int num_layers,
                   const float* const* w_ih_packed, const float* const* bias,
                   const float* const* w_hh_packed, const float* out_snake_alpha_exp,
                   const float* out_snake_inv_beta, float* workspace, int mode, void* stream) {
  return reslstm_impl(x, out, B, H, T, num_layers, w_ih_packed, bias, w_hh_packed, out_snake_alpha_exp,
                      out_snake_inv_beta, workspace, mode, stream, nullptr, nullptr, nullptr, nullptr);
}

int bc_reslstm_fwd_state(const float* x, float* out, int B, int H, int T, int num_layers,
                         const float* const* w_ih_packed, const float* const* bias,
                         const float* const* w_hh_packed, const float* out_snake_alpha_exp,
                         const float* out_snake_inv_beta, float* workspace, int mode, const float* h0,
                         const float* c0, float* hT, float* cT, void* stream) {
  if ((h0 == nullptr) != (c0 == nullptr) || (hT == nullptr) != (cT == nullptr)) return BC_ERR_ARG;
  return reslstm_impl(x, out, B, H, T, num_layers, w_ih_packed, bias, w_hh_packed, out_snake_alpha_exp,
                      out_snake_inv_beta, workspace, mode, stream, h0, c0, hT, cT);
}

// One direction of one LSTM layer over a ctb sequence: gx = W_ih lin + b (k = 1 conv, Cin input
// channels), then the recurrence into lout [H][T*B] (the persistent kernel, or one launch per step).
static int lstm_layer_dir(const float* lin, int Cin, const float* wih, const float* bias, const float* whh,
                          float* lout, float* gx, float* cst, float* const (&frag)[2], int B, int H, int T, int mode,
                          hipStream_t st, const float* h0, const float* c0, float* hT, float* cT, int* call_status,
                          void* psplit = nullptr) {
  const long long tb = (long long)T * B;
  if (!wih || !whh || !bias) return BC_ERR_ARG;
  ConvArgs a{};
  a.x = lin; a.w = wih; a.bias = bias; a.res = nullptr;
  a.osa = nullptr; a.osb = nullptr; a.y = gx; a.y2 = nullptr;
  a.xbs = Cin * tb; a.ybs = 4LL * H * tb; a.rbs = 0;  // one "batch item" (B = 1): the extents (debug-build checks)
  a.Cin = Cin; a.Tin = (int)tb; a.Cout = 4 * H; a.Nout = (int)tb;
  a.K = 1; a.s = 1; a.d = 1; a.pl = 0;
  a.yT = (int)tb; a.ostride = 1; a.ooff = 0; a.epi = 0;
  // W_ih is packed for the shape table's cfg (include/bigcodec.h), so the narrow-launch tiles do not apply here
  const int cfg = conv_select_cfg(4 * H, Cin, 1, 1, 1, mode);
  int rc;
  // (few columns, e.g. a streaming chunk: presplit_b walks every chunk of a 256-column tile in one workgroup, a fixed
  // ~220 us, so below 32 tiles the plain 322 launch, bit-identical, is faster; profiles/r04v_presplit_narrow.txt)
  const bool ps_size = tb >= 32 * 256 || g_lstm_presplit == 2;
  {  // (the launch timer: the pre-split launchers bracket their two kernels themselves)
    const double pfl = 2.0 * 4 * H * (double)Cin * tb, pby = 4.0 * ((double)Cin + 4.0 * H) * tb;
    if (psplit && g_lstm_presplit && cfg == 322 && ps_size && pw_presplit_ok(4 * H, Cin, tb)) {
      rc = pw_presplit_launch(a, psplit, st);  // same planes, scales and MFMA chains as cfg 322: bit-identical
    } else if (psplit && g_lstm_presplit && cfg == 122 && ps_size && pw_presplit_x6_ok(4 * H, Cin, tb)) {
      rc = pw_presplit_x6_launch(a, psplit, st);  // x6: the same planes and chains as cfg 122, 128-row tiles
    } else {
      char nm[160];
      if (conv_kernel_name(cfg, 1, 1, 1, nm, sizeof nm) < 0) snprintf(nm, sizeof nm, "conv cfg %d", cfg);
      LTScope lt(nm, pfl, pby, st);
      rc = conv_launch(a, 1, cfg, st);
    }
  }
  if (rc) return rc;
  if (lstm_use_seq(H, mode)) {  // workspace tail (cst onwards) holds the persistent kernel's flags + h fragments
    // algorithmic work: the recurrent GEMMs; bytes: gx read + the layer's output written
    LTScope lt(lstm_seq_kernel_name(H, lstm_planes(mode), B < 64 ? B : 64), 2.0 * 4 * H * (double)H * tb,
               4.0 * 5.0 * H * tb, st);
    return lstm_seq_launch(gx, reinterpret_cast<const unsigned short*>(whh), lout, cst, H, T, B, lstm_planes(mode), st,
                           h0, c0, hT, cT, call_status);
  }
  if (h0 || c0 || hT || cT) return BC_ERR_UNSUPPORTED;  // carried state: the persistent kernel only
  const bool fast = lstm_fast_ok(H);
  for (int t = 0; t < T; ++t) {
    rc = fast ? lstm_step_frag_launch(gx, whh, frag[(t + 1) & 1], frag[t & 1], lout, cst, H, B, T, t, st)
              : lstm_step_launch(gx, whh, lout, cst, H, B, T, t, st);
    if (rc) return rc;
  }
  return BC_OK;
}

static int reslstm_impl(const float* x, float* out, int B, int H, int T, int num_layers,
                        const float* const* w_ih_packed, const float* const* bias,
                        const float* const* w_hh_packed, const float* out_snake_alpha_exp,
                        const float* out_snake_inv_beta, float* workspace, int mode, void* stream,
                        const float* h0, const float* c0, float* hT, float* cT) {
  if (!x || !out || !w_ih_packed || !bias || !w_hh_packed || !workspace || B < 0 || H <= 0 ||
      H % 16 || T < 0 || num_layers <= 0 || mode < 0 || mode > 3)
    return BC_ERR_ARG;
  if ((out_snake_alpha_exp == nullptr) != (out_snake_inv_beta == nullptr)) return BC_ERR_ARG;
  hipStream_t st = S(stream);
  int* call_status = reinterpret_cast<int*>(workspace);  // workspace[0]: this call's timeout count
  if (hipMemsetAsync(call_status, 0, sizeof(int), st) != hipSuccess) return BC_ERR_LAUNCH;
  if (B == 0 || T == 0) return BC_OK;
  mode = lstm_mode(mode);
  const long long tb = (long long)T * B;
  if (tb > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  float* xt = workspace + LSTM_WS_STATUS_FLOATS;
  float* gx = xt + tb * H;
  float* ya = gx + tb * 4 * H;
  float* yb = ya + tb * H;
  float* cst = yb + tb * H;
  float* const frag[2] = {cst + (long long)H * B, cst + (long long)H * B + lstm_frag_floats(B, H)};
  int rc;
  {
    LTScope lt("btc_to_ctb_kernel", 0.0, 8.0 * H * tb, st);
    rc = btc_to_ctb_launch(x, xt, B, H, T, st);
  }
  if (rc) return rc;
  const float* lin = xt;
  float* lout = ya;
  for (int l = 0; l < num_layers; ++l) {
    const long long so = (long long)l * H * B;  // layer l's [H][B] state
    rc = lstm_layer_dir(lin, H, w_ih_packed[l], bias[l], w_hh_packed[l], lout, gx, cst, frag, B, H, T, mode, st,
                        h0 ? h0 + so : nullptr, c0 ? c0 + so : nullptr, hT ? hT + so : nullptr,
                        cT ? cT + so : nullptr, call_status, workspace + lstm_ws_head_floats(B, H, T));
    if (rc) return rc;
    lin = lout;
    lout = (lout == ya) ? yb : ya;
  }
  LTScope lt("ctb_to_btc_add_kernel", 0.0, 12.0 * H * tb, st);
  return ctb_to_btc_add_launch(lin, x, out_snake_alpha_exp, out_snake_inv_beta, out, B, H, T, st);
}

// Bidirectional ResLSTM (vq/module.py:150-152 with bidirectional=True: nn.LSTM(D, D / 2, bidirectional)):
// per layer the forward direction writes channels [0, H) of the layer output and the backward
// direction, run as the forward recurrence over the time-reversed input and reversed back, channels
// [H, 2H) (torch's concatenation order); every layer's input has D = 2H channels.
// workspace: status | xt [D][T*B] | gx [4H][T*B] | cat0, cat1 [D][T*B] | rin [D][T*B] | rout [H][T*B] |
// c [H][B] | hfrag x2 or the persistent kernel's region
long long bc_reslstm_bidir_workspace_floats(int B, int D, int T) {
  if (B < 0 || D <= 0 || D % 32 || T < 0) return -1;
  const int H = D / 2;
  const long long tb = (long long)T * B;
  const long long frag = 2 * lstm_frag_floats(B, H);
  const long long seq = lstm_seq_ok(H) ? lstm_seq_workspace_bytes(H, T) / 4 : 0;
  return LSTM_WS_STATUS_FLOATS + tb * D * 4 + tb * 4 * H + tb * H + (long long)H * B + (frag > seq ? frag : seq);
}

int bc_reslstm_bidir_fwd(const float* x, float* out, int B, int D, int T, int num_layers,
                         const float* const* w_ih_packed, const float* const* bias, const float* const* w_hh_packed,
                         const float* out_snake_alpha_exp, const float* out_snake_inv_beta, float* workspace, int mode,
                         void* stream) {
  if (!x || !out || !w_ih_packed || !bias || !w_hh_packed || !workspace || B < 0 || D <= 0 || D % 32 || T < 0 ||
      num_layers <= 0 || mode < 0 || mode > 3)
    return BC_ERR_ARG;
  if ((out_snake_alpha_exp == nullptr) != (out_snake_inv_beta == nullptr)) return BC_ERR_ARG;
  hipStream_t st = S(stream);
  int* call_status = reinterpret_cast<int*>(workspace);
  if (hipMemsetAsync(call_status, 0, sizeof(int), st) != hipSuccess) return BC_ERR_LAUNCH;
  if (B == 0 || T == 0) return BC_OK;
  mode = lstm_mode(mode);
  const int H = D / 2;
  const long long tb = (long long)T * B;
  if (tb > 0x7fffffffLL) return BC_ERR_UNSUPPORTED;
  float* xt = workspace + LSTM_WS_STATUS_FLOATS;
  float* gx = xt + tb * D;
  float* cat[2] = {gx + tb * 4 * H, gx + tb * 4 * H + tb * D};
  float* rin = cat[1] + tb * D;
  float* rout = rin + tb * D;
  float* cst = rout + tb * H;
  float* const frag[2] = {cst + (long long)H * B, cst + (long long)H * B + lstm_frag_floats(B, H)};
  int rc = btc_to_ctb_launch(x, xt, B, D, T, st);
  if (rc) return rc;
  const float* lin = xt;
  for (int l = 0; l < num_layers; ++l) {
    float* y = cat[l & 1];
    rc = lstm_layer_dir(lin, D, w_ih_packed[2 * l], bias[2 * l], w_hh_packed[2 * l], y, gx, cst, frag, B, H, T, mode,
                        st, nullptr, nullptr, nullptr, nullptr, call_status);
    if (rc) return rc;
    if ((rc = time_reverse_launch(lin, rin, D, T, B, st))) return rc;
    rc = lstm_layer_dir(rin, D, w_ih_packed[2 * l + 1], bias[2 * l + 1], w_hh_packed[2 * l + 1], rout, gx, cst, frag,
                        B, H, T, mode, st, nullptr, nullptr, nullptr, nullptr, call_status);
    if (rc) return rc;
    if ((rc = time_reverse_launch(rout, y + tb * H, H, T, B, st))) return rc;
    lin = y;
  }
  return ctb_to_btc_add_launch(lin, x, out_snake_alpha_exp, out_snake_inv_beta, out, B, D, T, st);
}

int bc_vq_prepare_codebook(const float* codebook, float* codebook_norm, float* codebook_sq,
                           int n_codes, int dim, void* stream) {
  if (!codebook || !codebook_norm || !codebook_sq || n_codes <= 0) return BC_ERR_ARG;
  if (dim != 8) return BC_ERR_UNSUPPORTED;
  return vq_prepare_launch(codebook, codebook_norm, codebook_sq, n_codes, S(stream));
}

int bc_vq_fwd(const float* z, const float* w_in, const float* b_in, const float* codebook,
              const float* codebook_norm, const float* codebook_sq, const float* w_out,
              const float* b_out, long long* idx, float* z_e_out, float* post_out, int B, int D,
              int T, int n_codes, int dim, void* stream) {
  if (!z || !w_in || !b_in || !codebook || !codebook_norm || !codebook_sq || !idx || B < 0 ||
      D <= 0 || T < 0 || n_codes <= 0)
    return BC_ERR_ARG;
  if (post_out && (!w_out || !b_out)) return BC_ERR_ARG;
  if (dim != 8) return BC_ERR_UNSUPPORTED;
  // algorithmic work: in_proj + the n_codes distances + out_proj per frame; bytes: z read, post written, indices
  const double fr = (double)B * T;
  LTScope lt("vq_fwd_kernel", fr * 2.0 * (D * 8.0 + 8.0 * n_codes + (post_out ? 8.0 * D : 0.0)),
             fr * (4.0 * D + (post_out ? 4.0 * D : 0.0) + 8.0 + (z_e_out ? 32.0 : 0.0)), S(stream));
  return vq_fwd_launch(z, w_in, b_in, codebook, codebook_norm, codebook_sq, w_out, b_out, idx,
                       z_e_out, post_out, B, D, T, n_codes, S(stream));
}

int bc_vq_argmin(const float* z_e, const float* codebook_norm, const float* codebook_sq,
                 long long* idx, long long N, int n_codes, int dim, void* stream) {
  if (!z_e || !codebook_norm || !codebook_sq || !idx || N < 0 || n_codes <= 0) return BC_ERR_ARG;
  if (dim != 8) return BC_ERR_UNSUPPORTED;
  return vq_argmin_launch(z_e, codebook_norm, codebook_sq, idx, N, n_codes, S(stream));
}

int bc_vq2emb(const long long* idx, long long idx_stride, const float* codebook,
              const float* w_out, const float* b_out, float* emb, long long N, int D, int n_codes,
              int dim, int accumulate, void* stream) {
  if (!idx || idx_stride <= 0 || !codebook || !emb || N < 0 || D <= 0 || n_codes <= 0)
    return BC_ERR_ARG;
  if ((w_out == nullptr) != (b_out == nullptr)) return BC_ERR_ARG;
  if (!w_out && D != dim) return BC_ERR_ARG;
  if (dim != 8) return BC_ERR_UNSUPPORTED;
  return vq2emb_launch(idx, idx_stride, codebook, w_out, b_out, emb, N, D, accumulate, S(stream));
}

int bc_fsq_fwd(const float* z, const float* w_in, const float* b_in, const float* w_out, const float* b_out,
               const float* consts, int* idx, float* post, int B, int D, int T, int d, void* stream) {
  return fsq_fwd_launch(z, w_in, b_in, w_out, b_out, consts, idx, post, B, D, T, d, S(stream));
}

int bc_stream_window(const float* x, long long x_batch_stride, long long x_row_stride, const float* ctx,
                     const float* snake_alpha_exp, const float* snake_inv_beta, float* win, float* ctx_out, int B, int C,
                     int n, int P, void* stream) {
  return stream_window_launch(x, x_batch_stride, x_row_stride, ctx, snake_alpha_exp, snake_inv_beta, win, ctx_out, B, C,
                              n, P, S(stream));
}

int bc_fsq_codes(const void* idx, int idx_bits, const int* levels, const float* w_out, const float* b_out,
                 float* post, int B, int D, int T, int d, void* stream) {
  return fsq_codes_launch(idx, idx_bits, levels, w_out, b_out, post, B, D, T, d, S(stream));
}

int bc_vq2emb_ct(const long long* idx, int nq, const float* codebooks, const float* w_out,
                 const float* b_out, float* emb, int B, int T, int D, int n_codes, int dim, void* stream) {
  if (dim != 8) return BC_ERR_UNSUPPORTED;
  return vq2emb_ct_launch(idx, nq, codebooks, w_out, b_out, emb, B, T, D, n_codes, S(stream));
}

int bc_resample_sinc(const float* x, float* y, const float* kern, int B, long long Lin, long long Lout,
                     long long y_pitch, int orig, int new_freq, int taps, int width, void* stream) {
  return resample_sinc_launch(x, y, kern, B, Lin, Lout, y_pitch, orig, new_freq, taps, width, S(stream));
}

int bc_rvq_update(float* residual, float* out, const float* q, long long n, int first,
                  void* stream) {
  if (!residual || !out || !q || n < 0) return BC_ERR_ARG;
  return rvq_update_launch(residual, out, q, n, first, S(stream));
}

int bc_btc_to_ctb(const float* x, float* y, int B, int C, int T, void* stream) {
  if (!x || !y || B < 0 || C < 0 || T < 0) return BC_ERR_ARG;
  return btc_to_ctb_launch(x, y, B, C, T, S(stream));
}

int bc_ctb_to_btc_add(const float* y, const float* skip, float* out, int B, int C, int T,
                      void* stream) {
  if (!y || !skip || !out || B < 0 || C < 0 || T < 0) return BC_ERR_ARG;
  return ctb_to_btc_add_launch(y, skip, nullptr, nullptr, out, B, C, T, S(stream));
}

int bc_conv1d_kernel_name(int cfg, int K, int stride, int dilation, char* buf, int buflen) {
  if (!buf || buflen <= 0) return -1;
  return conv_kernel_name(cfg, K, stride, dilation, buf, buflen);
}

int bc_resunit_kernel_name(int cfg, int C, int dilation, char* buf, int buflen) {
  if (!buf || buflen <= 0) return -1;
  return resunit_kernel_name(cfg, C, dilation, buf, buflen);
}

int bc_tanh_fwd(const float* x, float* y, long long n, void* stream) {
  if (!x || !y || n < 0) return BC_ERR_ARG;
  return tanh_launch(x, y, n, S(stream));
}

int bc_synth_clips(float* x, int B, long long T, long long clip0, void* stream) {
  if (!x || B < 0 || T < 0 || clip0 < 0) return BC_ERR_ARG;
  return synth_clips_launch(x, B, T, clip0, S(stream));
}

}  // extern "C"

// Diagnostics only (not part of include/bigcodec.h): run the unidirectional ResLSTM's input projection on the
// pre-split GEMM from 32 column tiles up (1, the default), at every size (2: the bit-identity test's small shapes)
// or on conv1d_x6_kernel (0); returns the previous setting.
extern "C" int bc_debug_set_lstm_presplit(int on) {
  const int old = g_lstm_presplit;
  g_lstm_presplit = on == 2 ? 2 : on ? 1 : 0;
  return old;
}

// ---- bounds-checked debug build (include/bigcodec.h) -------------------------------------------------------------
#ifdef BC_DEBUG
namespace bc {
__global__ void debug_selftest_kernel(int n) {
  if (!BC_DOK((int)(blockIdx.x * blockDim.x + threadIdx.x) >= n)) return;  // lanes < n fail on purpose
}
}  // namespace bc
BC_DEBUG_EXPORT(abi)
extern "C" {
int bc_dbg_fetch_conv1d(unsigned*);
int bc_dbg_fetch_conv1d_x6_p1(unsigned*);
int bc_dbg_fetch_conv1d_x6_p2(unsigned*);
int bc_dbg_fetch_conv1d_x6_p3(unsigned*);
int bc_dbg_fetch_conv1d_x6ra(unsigned*);
int bc_dbg_fetch_resunit_x6(unsigned*);
int bc_dbg_fetch_resunit_w16(unsigned*);
int bc_dbg_fetch_resunit_rr(unsigned*);
int bc_dbg_fetch_pw_presplit(unsigned*);
int bc_dbg_fetch_lstm_seq(unsigned*);
int bc_debug_status(unsigned* out) {
  if (!out) return BC_ERR_ARG;
  if (hipDeviceSynchronize() != hipSuccess) return BC_ERR_LAUNCH;
  out[0] = out[1] = 0;
  int (*const fetch[])(unsigned*) = {bc_dbg_fetch_conv1d, bc_dbg_fetch_conv1d_x6_p1, bc_dbg_fetch_conv1d_x6_p2, bc_dbg_fetch_conv1d_x6ra,
                                     bc_dbg_fetch_conv1d_x6_p3, bc_dbg_fetch_resunit_x6, bc_dbg_fetch_resunit_w16,
                                     bc_dbg_fetch_resunit_rr,
                                     bc_dbg_fetch_pw_presplit, bc_dbg_fetch_lstm_seq, bc_dbg_fetch_abi};
  for (auto f : fetch)
    if (f(out)) return BC_ERR_LAUNCH;
  return BC_OK;
}
int bc_debug_selftest(int n, void* stream) {
  if (n < 0 || n > 1 << 20) return BC_ERR_ARG;
  if (n == 0) return BC_OK;
  hipLaunchKernelGGL(debug_selftest_kernel, dim3((n + 255) / 256 + 1), dim3(256), 0, S(stream), n);
  BC_CHECK_LAUNCH();
  return BC_OK;
}
}
#else
extern "C" {
int bc_debug_status(unsigned* out) {
  if (out) out[0] = out[1] = 0;
  return BC_ERR_UNSUPPORTED;
}
int bc_debug_selftest(int n, void* stream) {
  (void)n, (void)stream;
  return BC_ERR_UNSUPPORTED;
}
}
#endif
