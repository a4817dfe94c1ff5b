// torch.ops.bigcodec.* — the C ABI of libbigcodec_hip.so (include/bigcodec.h) registered as PyTorch-ROCm
// custom operators ("A TORCH_LIBRARY(bigcodec, m) extension wraps them").
//
// Each op is functional (allocates its outputs with the caching allocator on the input's device) except
// the ones named with a trailing underscore, which mutate the arguments their schema marks (a!).  Every
// op runs stream-ordered on the CURRENT HIP stream of its input's device, checks device / dtype /
// contiguity / shape with TORCH_CHECK (-> Python RuntimeError, ValueError for bad values) and turns a
// nonzero ABI status into an error naming the entry point.  Only the HIP ("CUDA" dispatch key on
// PyTorch-ROCm) implementation lives here; the shape-only fake kernels for tracing / torch.compile /
// opcheck are registered in audiotokenization_amd/ops.py.
//
// Reference call chains replaced: see include/bigcodec.h, one comment per entry point.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "bigcodec.h"

namespace {

using at::Tensor;
using c10::optional;

const char* status_text(int rc) {
  switch (rc) {
    case 1: return "bad argument";
    case 2: return "HIP launch error";
    case 3: return "unsupported shape";
    default: return "error";
  }
}

void ok(int rc, const char* fn) { TORCH_CHECK(rc == 0, "bigcodec: ", fn, " failed: ", status_text(rc), " (code ", rc, ")"); }

void dev(const Tensor& t, const char* name, at::ScalarType st = at::kFloat) {
  TORCH_CHECK(t.is_cuda(), "bigcodec: ", name, " must be a HIP device tensor (there is no CPU path)");
  TORCH_CHECK(t.scalar_type() == st, "bigcodec: ", name, " must be ", st, ", got ", t.scalar_type());
  TORCH_CHECK(t.is_contiguous(), "bigcodec: ", name, " must be contiguous");
}

void same_device(const Tensor& a, const Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), "bigcodec: ", name, " is on ", b.device(), ", expected ", a.device());
}

const float* optf(const Tensor& ref, const optional<Tensor>& t, const char* name) {
  if (!t.has_value()) return nullptr;
  dev(*t, name);
  same_device(ref, *t, name);
  return t->data_ptr<float>();
}

const float* req(const Tensor& ref, const Tensor& t, const char* name) {
  dev(t, name);
  same_device(ref, t, name);
  return t.data_ptr<float>();
}

void check_coeffs(const optional<Tensor>& a, const optional<Tensor>& b, int64_t C, const char* what) {
  TORCH_CHECK(a.has_value() == b.has_value(), "bigcodec: ", what, ": alpha_exp and inv_beta come together");
  if (a.has_value()) TORCH_CHECK(a->numel() == C && b->numel() == C, "bigcodec: ", what, " coefficients must have ", C, " entries");
}

hipStream_t stream_of(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.get_device()).stream(); }

int i32(int64_t v, const char* name) {
  TORCH_CHECK_VALUE(v >= INT32_MIN && v <= INT32_MAX, "bigcodec: ", name, " = ", v, " does not fit int32");
  return static_cast<int>(v);
}

// ---- conv1d: WNConv1d / CausalConv1d (+ residual, tanh or next-Snake epilogue) ------------------------------
std::vector<Tensor> conv1d(const Tensor& x, const Tensor& w, const optional<Tensor>& bias,
                           const optional<Tensor>& residual, const optional<Tensor>& sa, const optional<Tensor>& sb,
                           int64_t cout, int64_t tout, int64_t k, int64_t stride, int64_t dilation, int64_t pad_left,
                           int64_t epilogue, int64_t cfg, bool dual) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() == 3, "bigcodec::conv1d: x must be (B, Cin, T)");
  TORCH_CHECK_VALUE(tout > 0 && cout > 0, "bigcodec::conv1d: Cout and Tout must be positive");
  TORCH_CHECK_VALUE(!dual || sa.has_value(), "bigcodec::conv1d: dual output needs the next Snake's coefficients");
  check_coeffs(sa, sb, cout, "conv1d out snake");
  const int64_t B = x.size(0);
  auto y = at::empty({B, cout, tout}, x.options());
  Tensor y2 = dual ? at::empty_like(y) : Tensor();
  if (residual.has_value())
    TORCH_CHECK_VALUE(residual->sizes() == y.sizes(), "bigcodec::conv1d: residual ", residual->sizes(), " != output ", y.sizes());
  if (bias.has_value()) TORCH_CHECK_VALUE(bias->numel() == cout, "bigcodec::conv1d: bias must have Cout entries");
  ok(bc_conv1d_fwd(x.data_ptr<float>(), req(x, w, "w_packed"), optf(x, bias, "bias"), optf(x, residual, "residual"),
                   optf(x, sa, "snake_alpha_exp"), optf(x, sb, "snake_inv_beta"), y.data_ptr<float>(),
                   dual ? y2.data_ptr<float>() : nullptr, i32(B, "B"), i32(x.size(1), "Cin"), i32(x.size(2), "T"),
                   i32(cout, "Cout"), i32(tout, "Tout"), i32(k, "K"), i32(stride, "stride"), i32(dilation, "dilation"),
                   i32(pad_left, "pad_left"), i32(epilogue, "epilogue"), i32(cfg, "cfg"), stream_of(x)),
     "bc_conv1d_fwd");
  if (dual) return {y, y2};
  return {y};
}

// ---- conv_transpose1d: WNConvTranspose1d / CausalConvTranspose1d (polyphase) -----------------------------------
std::vector<Tensor> conv_transpose1d(const Tensor& x, at::TensorList w_phases, const optional<Tensor>& bias,
                                     const optional<Tensor>& sa, const optional<Tensor>& sb, int64_t cout, int64_t tout,
                                     int64_t k, int64_t stride, int64_t padding, int64_t cfg, bool dual) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() == 3, "bigcodec::conv_transpose1d: x must be (B, Cin, T)");
  TORCH_CHECK_VALUE((int64_t)w_phases.size() == stride && stride > 0, "bigcodec::conv_transpose1d: one packed weight per phase");
  TORCH_CHECK_VALUE(tout > 0, "bigcodec::conv_transpose1d: Tout must be positive");
  TORCH_CHECK_VALUE(!dual || sa.has_value(), "bigcodec::conv_transpose1d: dual output needs the next Snake's coefficients");
  check_coeffs(sa, sb, cout, "conv_transpose1d out snake");
  std::vector<const float*> ph;
  for (const auto& w : w_phases) ph.push_back(req(x, w, "w_phases[r]"));
  const int64_t B = x.size(0);
  auto y = at::empty({B, cout, tout}, x.options());
  Tensor y2 = dual ? at::empty_like(y) : Tensor();
  // per-phase contiguous rows + one interleave pass (bc_convT1d_fwd_ws): the same values as the strided-store path
  const long long nws = bc_convT1d_workspace_floats(i32(B, "B"), i32(cout, "Cout"), i32(tout, "Tout"), i32(k, "K"),
                                                    i32(stride, "stride"), i32(padding, "padding"), dual ? 1 : 0);
  // nws < 0: a stride beyond the interleave's table (> 16): the strided-store path, no workspace
  auto ws = at::empty({(int64_t)(nws > 0 ? nws : 1)}, x.options());
  ok(bc_convT1d_fwd_ws(x.data_ptr<float>(), ph.data(), optf(x, bias, "bias"), optf(x, sa, "snake_alpha_exp"),
                       optf(x, sb, "snake_inv_beta"), y.data_ptr<float>(), dual ? y2.data_ptr<float>() : nullptr,
                       i32(B, "B"), i32(x.size(1), "Cin"), i32(x.size(2), "T"), i32(cout, "Cout"), i32(tout, "Tout"),
                       i32(k, "K"), i32(stride, "stride"), i32(padding, "padding"), i32(cfg, "cfg"),
                       nws >= 0 ? ws.data_ptr<float>() : nullptr, stream_of(x)),
     "bc_convT1d_fwd_ws");
  if (dual) return {y, y2};
  return {y};
}

// ---- resunit: a whole ResidualUnit in one launch -------------------------------------------------------------
std::vector<Tensor> resunit(const Tensor& x_raw, const optional<Tensor>& x_act, const optional<Tensor>& in_a,
                            const optional<Tensor>& in_b, const Tensor& w7, const optional<Tensor>& b7,
                            const Tensor& mid_a, const Tensor& mid_b, const Tensor& w1, const optional<Tensor>& b1,
                            const optional<Tensor>& out_a, const optional<Tensor>& out_b, int64_t dilation,
                            int64_t pad_left, int64_t cfg, bool dual) {
  dev(x_raw, "x_raw");
  TORCH_CHECK_VALUE(x_raw.dim() == 3, "bigcodec::resunit: x_raw must be (B, C, T)");
  const int64_t C = x_raw.size(1);
  TORCH_CHECK_VALUE(x_act.has_value() != in_a.has_value(),
                    "bigcodec::resunit: pass either the activated input x_act or the input Snake's coefficients");
  check_coeffs(in_a, in_b, C, "resunit in snake");
  check_coeffs(out_a, out_b, C, "resunit out snake");
  TORCH_CHECK_VALUE(mid_a.numel() == C && mid_b.numel() == C, "bigcodec::resunit: mid snake coefficients must have C entries");
  TORCH_CHECK_VALUE(!dual || out_a.has_value(), "bigcodec::resunit: dual output needs the next Snake's coefficients");
  if (x_act.has_value()) TORCH_CHECK_VALUE(x_act->sizes() == x_raw.sizes(), "bigcodec::resunit: x_act shape != x_raw shape");
  auto y = at::empty_like(x_raw);
  Tensor y2 = dual ? at::empty_like(x_raw) : Tensor();
  const int B = i32(x_raw.size(0), "B"), Ci = i32(C, "C"), T = i32(x_raw.size(2), "T");
  if (x_act.has_value()) {
    ok(bc_resunit_fwd(x_raw.data_ptr<float>(), req(x_raw, *x_act, "x_act"), req(x_raw, w7, "w7_packed"),
                      optf(x_raw, b7, "b7"), req(x_raw, mid_a, "mid_alpha_exp"), req(x_raw, mid_b, "mid_inv_beta"),
                      req(x_raw, w1, "w1_packed"), optf(x_raw, b1, "b1"), optf(x_raw, out_a, "out_alpha_exp"),
                      optf(x_raw, out_b, "out_inv_beta"), y.data_ptr<float>(), dual ? y2.data_ptr<float>() : nullptr, B,
                      Ci, T, i32(dilation, "dilation"), i32(pad_left, "pad_left"), i32(cfg, "cfg"), stream_of(x_raw)),
       "bc_resunit_fwd");
  } else {
    ok(bc_resunit_fwd_snake_in(x_raw.data_ptr<float>(), optf(x_raw, in_a, "in_alpha_exp"), optf(x_raw, in_b, "in_inv_beta"),
                               req(x_raw, w7, "w7_packed"), optf(x_raw, b7, "b7"), req(x_raw, mid_a, "mid_alpha_exp"),
                               req(x_raw, mid_b, "mid_inv_beta"), req(x_raw, w1, "w1_packed"), optf(x_raw, b1, "b1"),
                               optf(x_raw, out_a, "out_alpha_exp"), optf(x_raw, out_b, "out_inv_beta"),
                               y.data_ptr<float>(), dual ? y2.data_ptr<float>() : nullptr, B, Ci, T,
                               i32(dilation, "dilation"), i32(pad_left, "pad_left"), i32(cfg, "cfg"), stream_of(x_raw)),
       "bc_resunit_fwd_snake_in");
  }
  if (dual) return {y, y2};
  return {y};
}

// ---- activations --------------------------------------------------------------------------------------------
Tensor snake(const Tensor& x, const Tensor& a, const Tensor& ib) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() == 3, "bigcodec::snake: x must be (B, C, T)");
  TORCH_CHECK_VALUE(a.numel() == x.size(1) && ib.numel() == x.size(1), "bigcodec::snake: coefficients must have C entries");
  auto y = at::empty_like(x);
  ok(bc_snake_fwd(x.data_ptr<float>(), req(x, a, "alpha_exp"), req(x, ib, "inv_beta"), y.data_ptr<float>(),
                  i32(x.size(0), "B"), i32(x.size(1), "C"), x.size(2), stream_of(x)),
     "bc_snake_fwd");
  return y;
}

Tensor aa_snake(const Tensor& x, const Tensor& a, const Tensor& ib, const Tensor& fu, const Tensor& fd) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() == 3, "bigcodec::aa_snake: x must be (B, C, T)");
  TORCH_CHECK_VALUE(a.numel() == x.size(1) && ib.numel() == x.size(1), "bigcodec::aa_snake: coefficients must have C entries");
  TORCH_CHECK_VALUE(fu.numel() == 12 && fd.numel() == 12, "bigcodec::aa_snake: 12-tap filters");
  auto y = at::empty_like(x);
  ok(bc_aa_snake_fwd(x.data_ptr<float>(), req(x, a, "alpha_exp"), req(x, ib, "inv_beta"), req(x, fu, "up_filter"),
                     req(x, fd, "down_filter"), y.data_ptr<float>(), i32(x.size(0), "B"), i32(x.size(1), "C"),
                     i32(x.size(2), "T"), stream_of(x)),
     "bc_aa_snake_fwd");
  return y;
}

Tensor tanh_op(const Tensor& x) {
  dev(x, "x");
  auto y = at::empty_like(x);
  ok(bc_tanh_fwd(x.data_ptr<float>(), y.data_ptr<float>(), x.numel(), stream_of(x)), "bc_tanh_fwd");
  return y;
}

Tensor aa_snake_ex(const Tensor& x, const Tensor& a, const Tensor& ib, const Tensor& fu, const Tensor& fd,
                   int64_t up_ratio, int64_t down_ratio) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() == 3, "bigcodec::aa_snake_ex: x must be (B, C, T)");
  TORCH_CHECK_VALUE(a.numel() == x.size(1) && ib.numel() == x.size(1), "bigcodec::aa_snake_ex: coefficients must have C entries");
  const int T = i32(x.size(2), "T"), ru = i32(up_ratio, "up_ratio"), rd = i32(down_ratio, "down_ratio");
  const int ku = i32(fu.numel(), "up taps"), kd = i32(fd.numel(), "down taps");
  const long long Tout = bc_aa_snake_out_len(T, ru, rd, kd);
  TORCH_CHECK_VALUE(Tout >= 0, "bigcodec::aa_snake_ex: bad ratios");
  auto y = at::empty({x.size(0), x.size(1), (int64_t)Tout}, x.options());
  ok(bc_aa_snake_fwd_ex(x.data_ptr<float>(), req(x, a, "alpha_exp"), req(x, ib, "inv_beta"), req(x, fu, "up_filter"),
                        req(x, fd, "down_filter"), y.data_ptr<float>(), i32(x.size(0), "B"), i32(x.size(1), "C"), T, ru,
                        ku, rd, kd, stream_of(x)),
     "bc_aa_snake_fwd_ex");
  return y;
}

// ---- bidirectional ResLSTM: [y, status]; w_* hold [forward, backward] per layer ----------------------------------
std::vector<Tensor> reslstm_bidir(const Tensor& x, at::TensorList w_ih, at::TensorList bias, at::TensorList w_hh,
                                  const optional<Tensor>& sa, const optional<Tensor>& sb, int64_t mode) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() == 3, "bigcodec::reslstm_bidir: x must be (B, D, T)");
  const int64_t n = (int64_t)w_ih.size();
  TORCH_CHECK_VALUE(n > 0 && n % 2 == 0 && (int64_t)bias.size() == n && (int64_t)w_hh.size() == n,
                    "bigcodec::reslstm_bidir: w_ih / bias / w_hh hold [forward, backward] per layer");
  const int B = i32(x.size(0), "B"), D = i32(x.size(1), "D"), T = i32(x.size(2), "T");
  check_coeffs(sa, sb, D, "reslstm_bidir out snake");
  std::vector<const float*> pih, pb, phh;
  for (int64_t l = 0; l < n; ++l) {
    pih.push_back(req(x, w_ih[l], "w_ih_packed[l]"));
    pb.push_back(req(x, bias[l], "bias[l]"));
    phh.push_back(req(x, w_hh[l], "w_hh_packed[l]"));
  }
  const long long nws = bc_reslstm_bidir_workspace_floats(B, D, T);
  TORCH_CHECK_VALUE(nws >= 0, "bigcodec::reslstm_bidir: unsupported shape (D % 32 != 0)");
  auto ws = at::empty({std::max<long long>(nws, 64)}, x.options());
  auto y = at::empty_like(x);
  ok(bc_reslstm_bidir_fwd(x.data_ptr<float>(), y.data_ptr<float>(), B, D, T, (int)(n / 2), pih.data(), pb.data(),
                          phh.data(), optf(x, sa, "out_alpha_exp"), optf(x, sb, "out_inv_beta"), ws.data_ptr<float>(),
                          i32(mode, "mode"), stream_of(x)),
     "bc_reslstm_bidir_fwd");
  Tensor status = ws.narrow(0, 0, 1).view(at::kInt).clone();
  return {y, status};
}

// ---- ResLSTM: returns [y, status] (+ [hT, cT]); status = the call's int32 timeout count --------------------------
std::vector<Tensor> reslstm(const Tensor& x, at::TensorList w_ih, at::TensorList bias, at::TensorList w_hh,
                            const optional<Tensor>& sa, const optional<Tensor>& sb, int64_t mode,
                            const optional<Tensor>& h0, const optional<Tensor>& c0, bool return_state) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() == 3, "bigcodec::reslstm: x must be (B, H, T)");
  const int64_t L = (int64_t)w_ih.size();
  TORCH_CHECK_VALUE(L > 0 && (int64_t)bias.size() == L && (int64_t)w_hh.size() == L,
                    "bigcodec::reslstm: one w_ih / bias / w_hh per layer");
  TORCH_CHECK_VALUE(h0.has_value() == c0.has_value(), "bigcodec::reslstm: h0 and c0 come together");
  const int B = i32(x.size(0), "B"), H = i32(x.size(1), "H"), T = i32(x.size(2), "T");
  check_coeffs(sa, sb, H, "reslstm out snake");
  std::vector<const float*> pih, pb, phh;
  for (int64_t l = 0; l < L; ++l) {
    pih.push_back(req(x, w_ih[l], "w_ih_packed[l]"));
    pb.push_back(req(x, bias[l], "bias[l]"));
    phh.push_back(req(x, w_hh[l], "w_hh_packed[l]"));
  }
  const long long nws = bc_lstm_workspace_floats(B, H, T);
  TORCH_CHECK_VALUE(nws >= 0, "bigcodec::reslstm: unsupported shape");
  auto ws = at::empty({std::max<long long>(nws, 64)}, x.options());
  auto y = at::empty_like(x);
  const bool state = return_state || h0.has_value();
  Tensor hT, cT;
  if (state) {
    hT = at::empty({L, H, B}, x.options());
    cT = at::empty({L, H, B}, x.options());
    if (h0.has_value()) TORCH_CHECK_VALUE(h0->sizes() == hT.sizes() && c0->sizes() == cT.sizes(), "bigcodec::reslstm: h0 / c0 must be (layers, H, B)");
    ok(bc_reslstm_fwd_state(x.data_ptr<float>(), y.data_ptr<float>(), B, H, T, (int)L, pih.data(), pb.data(), phh.data(),
                            optf(x, sa, "out_alpha_exp"), optf(x, sb, "out_inv_beta"), ws.data_ptr<float>(),
                            i32(mode, "mode"), optf(x, h0, "h0"), optf(x, c0, "c0"), hT.data_ptr<float>(),
                            cT.data_ptr<float>(), stream_of(x)),
       "bc_reslstm_fwd_state");
  } else {
    ok(bc_reslstm_fwd(x.data_ptr<float>(), y.data_ptr<float>(), B, H, T, (int)L, pih.data(), pb.data(), phh.data(),
                      optf(x, sa, "out_alpha_exp"), optf(x, sb, "out_inv_beta"), ws.data_ptr<float>(), i32(mode, "mode"),
                      stream_of(x)),
       "bc_reslstm_fwd");
  }
  // include/bigcodec.h: ((int*)workspace)[0] is this call's timeout count; copied out so the (large)
  // workspace returns to the allocator now
  Tensor status = ws.narrow(0, 0, 1).view(at::kInt).clone();
  if (state) return {y, status, hT, cT};
  return {y, status};
}

// ---- quantizers ---------------------------------------------------------------------------------------------
std::vector<Tensor> vq_prepare_codebook(const Tensor& cb) {
  dev(cb, "codebook");
  TORCH_CHECK_VALUE(cb.dim() == 2, "bigcodec::vq_prepare_codebook: codebook must be (n_codes, dim)");
  auto norm = at::empty_like(cb);
  auto sq = at::empty({cb.size(0)}, cb.options());
  ok(bc_vq_prepare_codebook(cb.data_ptr<float>(), norm.data_ptr<float>(), sq.data_ptr<float>(), i32(cb.size(0), "n_codes"),
                            i32(cb.size(1), "dim"), stream_of(cb)),
     "bc_vq_prepare_codebook");
  return {norm, sq};
}

std::vector<Tensor> vq(const Tensor& z, const Tensor& w_in, const Tensor& b_in, const Tensor& cb, const Tensor& cbn,
                       const Tensor& cbsq, const Tensor& w_out, const Tensor& b_out, bool want_ze, bool want_post) {
  dev(z, "z");
  TORCH_CHECK_VALUE(z.dim() == 3, "bigcodec::vq: z must be (B, D, T)");
  TORCH_CHECK_VALUE(cb.dim() == 2 && cbn.sizes() == cb.sizes() && cbsq.numel() == cb.size(0), "bigcodec::vq: codebook shapes");
  const int64_t B = z.size(0), D = z.size(1), T = z.size(2), dim = cb.size(1);
  TORCH_CHECK_VALUE(w_in.numel() == dim * D && b_in.numel() == dim && w_out.numel() == D * dim && b_out.numel() == D,
                    "bigcodec::vq: projection shapes");
  auto idx = at::empty({B, T}, z.options().dtype(at::kLong));
  Tensor ze = want_ze ? at::empty({B, dim, T}, z.options()) : Tensor();
  Tensor post = want_post ? at::empty_like(z) : Tensor();
  ok(bc_vq_fwd(z.data_ptr<float>(), req(z, w_in, "w_in"), req(z, b_in, "b_in"), req(z, cb, "codebook"),
               req(z, cbn, "codebook_norm"), req(z, cbsq, "codebook_sq"), req(z, w_out, "w_out"), req(z, b_out, "b_out"),
               reinterpret_cast<long long*>(idx.data_ptr<int64_t>()), want_ze ? ze.data_ptr<float>() : nullptr,
               want_post ? post.data_ptr<float>() : nullptr, i32(B, "B"), i32(D, "D"), i32(T, "T"),
               i32(cb.size(0), "n_codes"), i32(dim, "dim"), stream_of(z)),
     "bc_vq_fwd");
  std::vector<Tensor> out{idx};
  if (want_ze) out.push_back(ze);
  if (want_post) out.push_back(post);
  return out;
}

Tensor vq_argmin(const Tensor& ze, const Tensor& cbn, const Tensor& cbsq) {
  dev(ze, "z_e");
  TORCH_CHECK_VALUE(ze.dim() == 2 && cbn.dim() == 2 && ze.size(1) == cbn.size(1), "bigcodec::vq_argmin: z_e (N, dim), codebook (n, dim)");
  auto idx = at::empty({ze.size(0)}, ze.options().dtype(at::kLong));
  ok(bc_vq_argmin(ze.data_ptr<float>(), req(ze, cbn, "codebook_norm"), req(ze, cbsq, "codebook_sq"), reinterpret_cast<long long*>(idx.data_ptr<int64_t>()),
                  ze.size(0), i32(cbn.size(0), "n_codes"), i32(cbn.size(1), "dim"), stream_of(ze)),
     "bc_vq_argmin");
  return idx;
}

// idx (..., nq) int64, column `column`; out (..., D)
void vq2emb_launch(const Tensor& idx, int64_t column, const Tensor& cb, const optional<Tensor>& w_out,
                   const optional<Tensor>& b_out, const Tensor& out, bool accumulate) {
  dev(idx, "idx", at::kLong);
  TORCH_CHECK_VALUE(idx.dim() >= 1 && column >= 0 && column < idx.size(-1), "bigcodec::vq2emb: column out of range");
  TORCH_CHECK_VALUE(w_out.has_value() == b_out.has_value(), "bigcodec::vq2emb: w_out and b_out come together");
  const int64_t nq = idx.size(-1), N = idx.numel() / nq;
  const int64_t D = w_out.has_value() ? w_out->size(0) : cb.size(1);
  TORCH_CHECK_VALUE(out.numel() == N * D, "bigcodec::vq2emb: output size");
  ok(bc_vq2emb(reinterpret_cast<const long long*>(idx.data_ptr<int64_t>()) + column, nq, req(idx, cb, "codebook"), optf(idx, w_out, "w_out"),
               optf(idx, b_out, "b_out"), out.data_ptr<float>(), N, i32(D, "D"), i32(cb.size(0), "n_codes"),
               i32(cb.size(1), "dim"), accumulate ? 1 : 0, stream_of(idx)),
     "bc_vq2emb");
}

Tensor vq2emb(const Tensor& idx, int64_t column, const Tensor& cb, const optional<Tensor>& w_out, const optional<Tensor>& b_out) {
  auto shape = idx.sizes().vec();
  shape.back() = w_out.has_value() ? w_out->size(0) : cb.size(1);
  auto out = at::empty(shape, idx.options().dtype(at::kFloat));
  vq2emb_launch(idx, column, cb, w_out, b_out, out, false);
  return out;
}

void vq2emb_add_(const Tensor& out, const Tensor& idx, int64_t column, const Tensor& cb, const optional<Tensor>& w_out,
                 const optional<Tensor>& b_out) {
  dev(out, "out");
  same_device(idx, out, "out");
  vq2emb_launch(idx, column, cb, w_out, b_out, out, true);
}

void rvq_update_(const Tensor& residual, const Tensor& out, const Tensor& q, bool first) {
  dev(residual, "residual");
  TORCH_CHECK_VALUE(out.sizes() == residual.sizes() && q.sizes() == residual.sizes(), "bigcodec::rvq_update_: shapes");
  ok(bc_rvq_update(residual.data_ptr<float>(), const_cast<float*>(req(residual, out, "out")), req(residual, q, "q"),
                   residual.numel(), first ? 1 : 0, stream_of(residual)),
     "bc_rvq_update");
}

Tensor vq2emb_ct(const Tensor& idx, const Tensor& cbs, const Tensor& w_out, const Tensor& b_out) {
  dev(idx, "idx", at::kLong);
  TORCH_CHECK_VALUE(idx.dim() == 3, "bigcodec::vq2emb_ct: idx must be (B, T, nq)");
  TORCH_CHECK_VALUE(cbs.dim() == 3 && w_out.dim() == 3 && b_out.dim() == 2, "bigcodec::vq2emb_ct: stacked parameters");
  const int64_t B = idx.size(0), T = idx.size(1), nq = idx.size(2), D = w_out.size(1);
  TORCH_CHECK_VALUE(nq <= cbs.size(0), "bigcodec::vq2emb_ct: more index columns than quantizers");
  auto out = at::empty({B, D, T}, idx.options().dtype(at::kFloat));
  ok(bc_vq2emb_ct(reinterpret_cast<const long long*>(idx.data_ptr<int64_t>()), i32(nq, "nq"), req(idx, cbs, "codebooks"), req(idx, w_out, "w_out"),
                  req(idx, b_out, "b_out"), out.data_ptr<float>(), i32(B, "B"), i32(T, "T"), i32(D, "D"),
                  i32(cbs.size(1), "n_codes"), i32(cbs.size(2), "dim"), stream_of(idx)),
     "bc_vq2emb_ct");
  return out;
}

std::vector<Tensor> stream_window(const Tensor& x, const optional<Tensor>& ctx, const optional<Tensor>& a,
                                  const optional<Tensor>& ib, int64_t P) {
  TORCH_CHECK(x.is_cuda(), "bigcodec: x must be a HIP device tensor (there is no CPU path)");
  TORCH_CHECK_VALUE(x.scalar_type() == at::kFloat && x.dim() == 3 && x.stride(2) == 1,
                    "bigcodec::stream_window: x must be a (B, C, n) float32 tensor with unit time stride");
  const int64_t B = x.size(0), C = x.size(1), n = x.size(2);
  TORCH_CHECK_VALUE(P >= 0 && n >= 1, "bigcodec::stream_window: P >= 0 and a non-empty chunk");
  check_coeffs(a, ib, C, "stream_window");
  if (ctx) TORCH_CHECK_VALUE(ctx->sizes() == at::IntArrayRef({B, C, P}), "bigcodec::stream_window: ctx must be (B, C, P)");
  auto win = at::empty({B, C, P + n}, x.options());
  auto nctx = at::empty({B, C, P}, x.options());
  ok(bc_stream_window(x.data_ptr<float>(), B > 1 ? x.stride(0) : C * x.stride(1), C > 1 ? x.stride(1) : n,
                      optf(x, ctx, "ctx"), optf(x, a, "alpha_exp"), optf(x, ib, "inv_beta"), win.data_ptr<float>(),
                      nctx.data_ptr<float>(), i32(B, "B"), i32(C, "C"), i32(n, "n"), i32(P, "P"), stream_of(x)),
     "bc_stream_window");
  return {win, nctx};
}

Tensor fsq_codes(const Tensor& idx, const Tensor& w_out, const Tensor& b_out, at::IntArrayRef levels) {
  TORCH_CHECK_VALUE(idx.is_cuda() && (idx.scalar_type() == at::kInt || idx.scalar_type() == at::kLong) &&
                        idx.is_contiguous(),
                    "bigcodec::fsq_codes: idx must be a contiguous int32 / int64 device tensor");
  TORCH_CHECK_VALUE(idx.dim() == 2, "bigcodec::fsq_codes: idx must be (B, T)");
  const int64_t B = idx.size(0), T = idx.size(1), d = (int64_t)levels.size(), D = b_out.numel();
  TORCH_CHECK_VALUE(d >= 1 && d <= 8 && w_out.numel() == D * d, "bigcodec::fsq_codes: parameter shapes");
  std::vector<int> lv(levels.begin(), levels.end());
  auto post = at::empty({B, D, T}, idx.options().dtype(at::kFloat));
  ok(bc_fsq_codes(idx.data_ptr(), idx.scalar_type() == at::kLong ? 64 : 32, lv.data(), req(idx, w_out, "w_out"),
                  req(idx, b_out, "b_out"), post.data_ptr<float>(), i32(B, "B"), i32(D, "D"), i32(T, "T"), (int)d,
                  stream_of(idx)),
     "bc_fsq_codes");
  return post;
}

std::vector<Tensor> fsq(const Tensor& z, const Tensor& w_in, const Tensor& b_in, const Tensor& w_out, const Tensor& b_out,
                        const Tensor& consts) {
  dev(z, "z");
  TORCH_CHECK_VALUE(z.dim() == 3, "bigcodec::fsq: z must be (B, D, T)");
  const int64_t B = z.size(0), D = z.size(1), T = z.size(2), d = b_in.numel();
  TORCH_CHECK_VALUE(w_in.numel() == d * D && w_out.numel() == D * d && b_out.numel() == D && consts.numel() == 5 * d,
                    "bigcodec::fsq: parameter shapes");
  auto post = at::empty_like(z);
  auto idx = at::empty({B, T}, z.options().dtype(at::kInt));
  ok(bc_fsq_fwd(z.data_ptr<float>(), req(z, w_in, "w_in"), req(z, b_in, "b_in"), req(z, w_out, "w_out"),
                req(z, b_out, "b_out"), req(z, consts, "consts"), idx.data_ptr<int>(), post.data_ptr<float>(), i32(B, "B"),
                i32(D, "D"), i32(T, "T"), i32(d, "d"), stream_of(z)),
     "bc_fsq_fwd");
  return {post, idx};
}

// ---- ingest / synthetic input -------------------------------------------------------------------------------
Tensor resample_sinc(const Tensor& x, const Tensor& kern, int64_t lout, int64_t pitch, int64_t orig, int64_t new_freq,
                     int64_t taps, int64_t width) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() >= 1 && pitch >= lout && lout >= 0, "bigcodec::resample_sinc: pitch >= Lout >= 0");
  const int64_t n = x.size(-1), rows = n ? x.numel() / n : 0;
  auto shape = x.sizes().vec();
  shape.back() = pitch;
  auto y = pitch > lout ? at::zeros(shape, x.options()) : at::empty(shape, x.options());
  ok(bc_resample_sinc(x.data_ptr<float>(), y.data_ptr<float>(), req(x, kern, "kern"), i32(rows, "rows"), n, lout, pitch,
                      i32(orig, "orig"), i32(new_freq, "new_freq"), i32(taps, "taps"), i32(width, "width"), stream_of(x)),
     "bc_resample_sinc");
  return y;
}

void synth_clips_(const Tensor& x, int64_t clip0) {
  dev(x, "x");
  TORCH_CHECK_VALUE(x.dim() >= 1, "bigcodec::synth_clips_: x must be (B, ..., T)");
  const int64_t T = x.size(-1), B = T ? x.numel() / T : 0;
  ok(bc_synth_clips(x.data_ptr<float>(), i32(B, "B"), T, clip0, stream_of(x)), "bc_synth_clips");
}

// Every op runs under a device guard of its first tensor argument (the data tensor), so the C ABI's launches
// and the op's allocations land on that tensor's device even when it is not the current one (the ABI launches
// on the current HIP device; c10 reports these tensors as "cuda", hence the masquerading guard).
template <auto F>
struct Guarded;
template <typename R, typename First, typename... Rest, R (*F)(First, Rest...)>
struct Guarded<F> {
  static R call(First first, Rest... rest) {
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(first.device());
    return F(first, rest...);
  }
};

}  // namespace

TORCH_LIBRARY(bigcodec, m) {
  m.def("conv1d(Tensor x, Tensor w_packed, Tensor? bias, Tensor? residual, Tensor? snake_alpha_exp, "
        "Tensor? snake_inv_beta, int cout, int tout, int kernel_size, int stride, int dilation, int pad_left, "
        "int epilogue, int cfg, bool dual) -> Tensor[]");
  m.def("conv_transpose1d(Tensor x, Tensor[] w_phases, Tensor? bias, Tensor? snake_alpha_exp, Tensor? snake_inv_beta, "
        "int cout, int tout, int kernel_size, int stride, int padding, int cfg, bool dual) -> Tensor[]");
  m.def("resunit(Tensor x_raw, Tensor? x_act, Tensor? in_alpha_exp, Tensor? in_inv_beta, Tensor w7_packed, Tensor? b7, "
        "Tensor mid_alpha_exp, Tensor mid_inv_beta, Tensor w1_packed, Tensor? b1, Tensor? out_alpha_exp, "
        "Tensor? out_inv_beta, int dilation, int pad_left, int cfg, bool dual) -> Tensor[]");
  m.def("snake(Tensor x, Tensor alpha_exp, Tensor inv_beta) -> Tensor");
  m.def("aa_snake(Tensor x, Tensor alpha_exp, Tensor inv_beta, Tensor up_filter, Tensor down_filter) -> Tensor");
  m.def("aa_snake_ex(Tensor x, Tensor alpha_exp, Tensor inv_beta, Tensor up_filter, Tensor down_filter, int up_ratio, "
        "int down_ratio) -> Tensor");
  m.def("tanh(Tensor x) -> Tensor");
  m.def("reslstm(Tensor x, Tensor[] w_ih_packed, Tensor[] bias, Tensor[] w_hh_packed, Tensor? out_alpha_exp, "
        "Tensor? out_inv_beta, int mode, Tensor? h0, Tensor? c0, bool return_state) -> Tensor[]");
  m.def("reslstm_bidir(Tensor x, Tensor[] w_ih_packed, Tensor[] bias, Tensor[] w_hh_packed, Tensor? out_alpha_exp, "
        "Tensor? out_inv_beta, int mode) -> Tensor[]");
  m.def("vq_prepare_codebook(Tensor codebook) -> Tensor[]");
  m.def("vq(Tensor z, Tensor w_in, Tensor b_in, Tensor codebook, Tensor codebook_norm, Tensor codebook_sq, "
        "Tensor w_out, Tensor b_out, bool want_ze, bool want_post) -> Tensor[]");
  m.def("vq_argmin(Tensor z_e, Tensor codebook_norm, Tensor codebook_sq) -> Tensor");
  m.def("vq2emb(Tensor idx, int column, Tensor codebook, Tensor? w_out, Tensor? b_out) -> Tensor");
  m.def("vq2emb_add_(Tensor(a!) out, Tensor idx, int column, Tensor codebook, Tensor? w_out, Tensor? b_out) -> ()");
  m.def("rvq_update_(Tensor(a!) residual, Tensor(b!) out, Tensor q, bool first) -> ()");
  m.def("vq2emb_ct(Tensor idx, Tensor codebooks, Tensor w_out, Tensor b_out) -> Tensor");
  m.def("fsq(Tensor z, Tensor w_in, Tensor b_in, Tensor w_out, Tensor b_out, Tensor consts) -> Tensor[]");
  m.def("fsq_codes(Tensor idx, Tensor w_out, Tensor b_out, int[] levels) -> Tensor");
  m.def("stream_window(Tensor x, Tensor? ctx, Tensor? alpha_exp, Tensor? inv_beta, int P) -> Tensor[]");
  m.def("resample_sinc(Tensor x, Tensor kern, int lout, int pitch, int orig, int new_freq, int taps, int width) -> Tensor");
  m.def("synth_clips_(Tensor(a!) x, int clip0) -> ()");
}

TORCH_LIBRARY_IMPL(bigcodec, CUDA, m) {
  m.impl("conv1d", &Guarded<&conv1d>::call);
  m.impl("conv_transpose1d", &Guarded<&conv_transpose1d>::call);
  m.impl("resunit", &Guarded<&resunit>::call);
  m.impl("snake", &Guarded<&snake>::call);
  m.impl("aa_snake", &Guarded<&aa_snake>::call);
  m.impl("tanh", &Guarded<&tanh_op>::call);
  m.impl("aa_snake_ex", &Guarded<&aa_snake_ex>::call);
  m.impl("reslstm", &Guarded<&reslstm>::call);
  m.impl("reslstm_bidir", &Guarded<&reslstm_bidir>::call);
  m.impl("vq_prepare_codebook", &Guarded<&vq_prepare_codebook>::call);
  m.impl("vq", &Guarded<&vq>::call);
  m.impl("vq_argmin", &Guarded<&vq_argmin>::call);
  m.impl("vq2emb", &Guarded<&vq2emb>::call);
  m.impl("vq2emb_add_", &Guarded<&vq2emb_add_>::call);
  m.impl("rvq_update_", &Guarded<&rvq_update_>::call);
  m.impl("vq2emb_ct", &Guarded<&vq2emb_ct>::call);
  m.impl("fsq", &Guarded<&fsq>::call);
  m.impl("fsq_codes", &Guarded<&fsq_codes>::call);
  m.impl("stream_window", &Guarded<&stream_window>::call);
  m.impl("resample_sinc", &Guarded<&resample_sinc>::call);
  m.impl("synth_clips_", &Guarded<&synth_clips_>::call);
}
