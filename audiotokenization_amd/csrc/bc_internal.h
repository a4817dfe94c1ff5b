// Host-side launchers shared between the kernel translation units and the C ABI (abi.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace bc {
struct ConvArgs {
  const float* x;      // input [B][Cin][Tin] (already activated: the Snake runs in the producer)
  const float* w;      // packed folded weights
  const float* bias;   // [Cout] or nullptr
  const float* res;    // residual, same indexing as y, or nullptr
  const float* osa;    // epilogue Snake alpha_exp [Cout] or nullptr
  const float* osb;    // epilogue Snake inv_beta [Cout]
  float* y;            // output (raw, or snake'd when osa != nullptr and y2 == nullptr)
  float* y2;           // optional second output = snake(raw) (dual epilogue)
  long long xbs, ybs, rbs;
  int Cin, Tin, Cout, Nout;
  int K, s, d, pl;
  int yT, ostride, ooff;
  int epi;             // 0 none, 1 tanh
  // phase decomposition of a strided conv (x6 kernel, cfg >= 1000): the kernel runs the stride-1
  // conv over ps * cin0 phase channels ci' = ci * ps + r, x_r[ci][m] = x[ci][m * ps + r - pl]
  int ps;              // 0: off
  int cin0;            // real input channels when ps != 0
  const float* wsc;    // h3 kernels: 1 / weight scale per output row (stored after the packed planes)
  int dbg;             // BC_X6_DEBUG timing experiments (x6 kernel): 1 no A copies, 2 no B loads, 4 no B stores, 8 no epilogue, 16 s_setprio(1) around the MFMAs, 32 no Snake on load (conv1d_x6_body)
  // filled by conv_launch
  int vec;             // 16-byte epilogue accesses allowed (conv_epilogue_vec_ok)
  int nchunks, win, bstage, astage;
  int bpitch;          // x6 kernel: bytes per B-tile column per plane (64: swizzled, stride 1; 80: strided)
  int prio;            // x6 kernel, 16-wave tile: s_setprio(1) for waves 8-15 for the whole launch (BC_X6_PRIO, A/B)
  const float* isa;    // conv1d_x6_body<..., SIN>: Snake applied to the staged input, alpha_exp [Cin] / inv_beta [Cin]
  const float* isb;
  int sin_lds;         // SIN 2: byte offset of the [isa][isb] table in the kernel's dynamic LDS
  float inv_win;
  int ntm, ntn, nwg;
};
// mode 0: fp32 MFMA kernel (cfg 0..19); mode 1: fp32-accurate 3xbf16 kernel (cfg 100..) where the
// shape suits it, else the fp32 kernel; mode 2: plain bf16 products (cfg 200..), else fp32.
int conv_select_cfg(int Cout, int Cin, int K, int stride, int dilation, int mode = 0);
bool conv_cfg_valid(int cfg_id);
int x6_select_cfg(int Cout, int Cin, int K, int s, int d, int planes);
int x6_narrow_cfg(int cfg, int Cout, int K, int s, int d, int planes, int B, int Tout, int cus);
bool x6_cfg_valid(int cfg);
long long x6_packed_bytes(int Cout, int Cin, int K, int cfg);
void x6_pack_weight(const float* w, unsigned short* out, int Cout, int Cin, int K, int cfg);
int x6_launch(ConvArgs& a, int B, int cfg, hipStream_t st);
// x6 convs with register-resident weight fragments on the 8-wave 192 x 256 tile (conv1d_x6ra.hip): the launches
// x6_launch routes from cfg 120 (the multi-tap stride-1 convs incl. the phase-decomposed strided ones)
bool x6ra_applies(int K, int s, int d, int ps);
const char* x6ra_kernel_name(bool b4);
int x6ra_launch(ConvArgs& a, int B, hipStream_t st);
int x6_kernel_name(int cfg, int K, int s, int d, char* buf, int n);
int conv_kernel_name(int cfg_id, int K, int s, int d, char* buf, int n);
int resunit_kernel_name(int cfg, int C, int d, char* buf, int n);
int resunit_rr_kernel_name(int C, int d, char* buf, int n);
long long conv_packed_floats(int Cout, int Cin, int K, int cfg_id);
void conv_pack_weight(const float* w, float* out, int Cout, int Cin, int K, int cfg_id);
int conv_launch(ConvArgs& a, int B, int cfg_id, hipStream_t st);

int resunit_select_cfg(int C, int d, int mode);
bool resunit_cfg_ok(int cfg, int C, int d);
// ConvTranspose1d: the phase rows of bc_convT1d_fwd_ws's workspace -> the output in order (elementwise.hip)
constexpr int CONVT_MAX_STRIDE = 16;
struct ConvTInterleave {
  int s, p;
  int q_lo[CONVT_MAX_STRIDE];
};
int convT_interleave_launch(const float* ph, const float* ph2, float* y, float* y2, int B, int Cout, int Tout, int Q4,
                            const ConvTInterleave& il, hipStream_t st);
// pointwise GEMM with a pre-split B operand (pw_presplit.hip; the ResLSTM input projection in h3)
long long pw_presplit_bytes(int Cin, long long N);
bool pw_presplit_ok(int Cout, int Cin, long long N);
int pw_presplit_launch(ConvArgs& a, void* ws, hipStream_t st);
bool pw_presplit_x6_ok(int Cout, int Cin, long long N);  // the x6 variant (128 x 256 tile over cfg-122 weights)
int pw_presplit_x6_launch(ConvArgs& a, void* ws, hipStream_t st);
// one-launch ResidualUnit at C = 192 on the 16-wave 192 x 256 tile (resunit_w16.hip; x6 cfg 122, bf16 cfg 222)
bool resunit_w16_ok(int C, int d, int P);
int resunit_w16_launch(ConvArgs& a, ConvArgs& e, const float* w1, const float* s2a, const float* s2b, int B, int P,
                       hipStream_t st);
int resunit_launch(const float* x_raw, const float* x_act, const float* w7, const float* b7, const float* s2a,
                   const float* s2b, const float* w1, const float* b1, const float* osa, const float* osb,
                   float* y, float* y2, int B, int C, int T, int d, int pl, int cfg, hipStream_t st,
                   const float* isa = nullptr, const float* isb = nullptr);

bool resunit_rr_ok(int C, int d);
int resunit_rr_launch(const float* x_raw, const float* x_act, const float* w7, const float* b7, const float* s2a,
                      const float* s2b, const float* w1, const float* b1, const float* osa, const float* osb, float* y,
                      float* y2, int B, int C, int T, int d, int pl, hipStream_t st, const float* isa,
                      const float* isb);

int snake_launch(const float* x, const float* sa, const float* sb, float* y, int B, int C,
                 long long T, hipStream_t st);
int stream_window_launch(const float* x, long long xbs, long long xT, const float* ctx, const float* sa, const float* sb,
                         float* win, float* ctx_out, int B, int C, int n, int P, hipStream_t st);
int aa_snake_launch(const float* x, const float* sa, const float* sb, const float* fu,
                    const float* fd, float* y, int B, int C, int T, hipStream_t st);
int btc_to_ctb_launch(const float* x, float* y, int B, int C, int T, hipStream_t st);
int ctb_to_btc_add_launch(const float* y, const float* skip, const float* sa, const float* sb,
                          float* out, int B, int C, int T, hipStream_t st);
int synth_clips_launch(float* x, int B, long long T, long long clip0, hipStream_t st);
int tanh_launch(const float* x, float* y, long long n, hipStream_t st);
int time_reverse_launch(const float* x, float* y, int C, int T, int B, hipStream_t st);
long long aa_snake_out_len(int T, int ru, int rd, int kd);
int aa_snake_gen_launch(const float* x, const float* sa, const float* sb, const float* fu, const float* fd, float* y,
                        int B, int C, int T, int ru, int ku, int rd, int kd, hipStream_t st);

bool lstm_fast_ok(int H);
void lstm_pack_hh2(const float* w, float* out, int H);
int lstm_step_frag_launch(const float* gx, const float* whh_p2, const float* hin, float* hout,
                          float* y, float* cst, int H, int B, int T, int t, hipStream_t st);
void lstm_pack_hh(const float* w, float* out, int H);
bool lstm_seq_ok(int H);
long long lstm_seq_packed_bytes(int H, int planes);
void lstm_seq_pack(const float* w, unsigned short* out, int H, int planes);
long long lstm_seq_workspace_bytes(int H, int T);
int lstm_seq_launch(const float* gx, const unsigned short* whh, float* y, void* ws, int H, int T, int Btot,
                    int planes, hipStream_t st, const float* h0 = nullptr, const float* c0 = nullptr,
                    float* hT = nullptr, float* cT = nullptr,
                    int* call_status = nullptr);
int lstm_seq_read_status(int reset);
int lstm_step_launch(const float* gx, const float* whh_p, float* y, float* cst, int H, int B,
                     int T, int t, hipStream_t st);

int mfma_probe_launch(float* out, int nwg, int iters, hipStream_t st);

// Launch timer (bc_launch_timer_*, abi.hip): LTScope brackets the launches of its lifetime with HIP events on `st`
// while the timer is enabled (a no-op otherwise).
struct LTScope {
  int idx;
  hipStream_t st_ = nullptr;
  LTScope(const char* name, double flops, double bytes, hipStream_t st);
  ~LTScope();
};
const char* lstm_seq_kernel_name(int H, int planes, int nb);  // the variant lstm_seq_launch runs for nb clips

int vq_prepare_launch(const float* cb, float* cbn, float* csq, int n, hipStream_t st);
int vq_fwd_launch(const float* z, const float* w_in, const float* b_in, const float* cb,
                  const float* cbn, const float* csq, const float* w_out, const float* b_out,
                  long long* idx, float* ze_out, float* post, int B, int D, int T, int ncodes,
                  hipStream_t st);
int vq_argmin_launch(const float* ze, const float* cbn, const float* csq, long long* idx,
                     long long N, int ncodes, hipStream_t st);
int resample_sinc_launch(const float* x, float* y, const float* kern, int B, long long Lin, long long Lout,
                         long long ypitch, int orig, int nw, int K, int width, hipStream_t st);
int fsq_fwd_launch(const float* z, const float* w_in, const float* b_in, const float* w_out, const float* b_out,
                   const float* consts, int* idx, float* post, int B, int D, int T, int nd, hipStream_t st);
int fsq_codes_launch(const void* idx, int idx_bits, const int* levels, const float* w_out, const float* b_out,
                     float* post, int B, int D, int T, int nd, hipStream_t st);
int vq2emb_ct_launch(const long long* idx, int nq, const float* cb, const float* w_out, const float* b_out,
                     float* emb, int B, int T, int D, int n_codes, hipStream_t st);
int vq2emb_launch(const long long* idx, long long idx_stride, const float* cb, const float* w_out,
                  const float* b_out, float* emb, long long N, int D, int accumulate,
                  hipStream_t st);
int rvq_update_launch(float* residual, float* out, const float* q, long long n, int first,
                      hipStream_t st);
}  // namespace bc
