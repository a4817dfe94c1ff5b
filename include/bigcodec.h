/*
 * bigcodec.h — C ABI of libbigcodec_hip.so, the MI355X (gfx950) BigCodec tokenization hot path.
 *
 * The reference (hoyso48/AudioTokenization, BigCodec_SSL/) is pure PyTorch and has no FFI: its
 * boundary is the nn.Module call surface of vq/codec_encoder.py, vq/codec_decoder.py and the
 * modules they compose.  Each entry point below replaces one aten call chain behind one of those
 * modules (cited per function).  The Python package audiotokenization_amd binds them with ctypes
 * (INTEGRATION.md shows the binding) and mirrors the reference modules on top.
 *
 * Conventions
 *   - every pointer argument named x/y/z/... is DEVICE memory (fp32 unless stated) and contiguous in
 *     the stated layout; pointers named *_host are host memory;
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream); all launches are
 *     stream-ordered and asynchronous; no function allocates, frees or synchronises;
 *   - return value: 0 = ok, 1 = bad argument, 2 = HIP launch error, 3 = unsupported shape.
 *   - activations are [B][C][T] (batch, channel, time) as in the reference's Conv1d tensors.
 */
#ifndef BIGCODEC_H
#define BIGCODEC_H

#ifdef __cplusplus
extern "C" {
#endif

#define BC_ABI_VERSION 17

int bc_abi_version(void);
/* bc_build_digest: sha256 (64 hex characters) of the sources, headers and compiler flags this library was built
 * from (ABI 16).  build_lib.py compiles it in and rebuilds when it differs from the tree's; bench.py reports a
 * committed PMC profile's traffic only when the profile was taken on a library with the running one's digest. */
const char* bc_build_digest(void);

/* ---- Conv1d (weight-normed, fused residual / tanh / next-Snake epilogue) --------------------------
 * Replaces: F.pad + conv1d of CausalConv1d.forward (vq/module.py:45-48) and weight_norm(nn.Conv1d)
 * (vq/module.py:59-65), followed by ResidualUnit's `x + ...` (vq/module.py:88-89) when
 * residual != NULL, by nn.Tanh (vq/codec_decoder.py:80) when epilogue == 1, and by the SnakeBeta of
 * the NEXT Activation1d (vq/activations.py:107-118) when out_snake_alpha_exp != NULL:
 *   v[b,co,n] = residual[b,co,n] + bias[co] + sum_{ci,k} W[co,ci,k] * x[b,ci, n*stride + k*dilation - pad_left]
 *   y = snake_co(v) (y2 == NULL)   or   y = v, y2 = snake_co(v) (dual output)   or   y = v / tanh(v)
 * Out-of-range input samples read as 0 (zero padding).  Non-causal: pad_left = padding; causal:
 * pad_left = (K - stride) * dilation (vq/module.py:43).  The input x is the already-activated
 * tensor (the Snake that precedes every reference conv runs in the producer's epilogue or in
 * bc_snake_fwd).  W is the FOLDED weight g*v/||v|| [Cout][Cin][K] packed by bc_conv1d_pack for
 * cfg = bc_conv1d_select_cfg(Cout, Cin, K, stride, dilation, mode) (any other valid tile id also
 * runs — tuning — with weights packed for that same cfg; a tile the shape does not fit returns 3).
 * mode 0: fp32 MFMA (v_mfma_f32_16x16x4_f32).  mode 1 (the package default): fp32-accurate "x6" MFMA — both operands
 * split exactly into three bf16 terms, six bf16 products per pair accumulated in fp32 — for the
 * shapes where it applies (Cin >= 16), else the fp32 kernel.  Its error against fp64 is at or below
 * the fp32 kernel's.  mode 2: plain bf16 products with fp32 accumulation (one MFMA
 * per pair; BASELINE config 5's "bf16 encoder conv stack"; activations stay fp32 in memory) where
 * Cin >= 16, else fp32.  bc_reslstm_fwd runs mode 2 as mode 3 (the recurrence stays fp32-class; its
 * input projection is packed with cfg = bc_conv1d_select_cfg(..., 3)).
 * mode 3 ("h3", opt-in; 22-bit operands, narrower than the reference's fp32): block-scaled 2 x fp16 split — each operand block is
 * scaled by a power of two from its maximum (weights per output row, packed by bc_conv1d_pack;
 * activations per staged 32-channel chunk) and split v*S = hi + lo (two fp16 terms, 22 significant
 * bits); a*b accumulates hi*hi + hi*lo + lo*hi in fp32 on v_mfma_f32_16x16x32_f16 (the dropped lo*lo
 * term is below 2^-22 |ab|), 3 MFMAs per pair, where Cin >= 16, else fp32.  Error against fp64 at or
 * below the native fp32 kernel's.
 * out_snake_alpha_exp[c] = exp(alpha[c]); out_snake_inv_beta[c] = 1/(exp(beta[c]) + 1e-9).
 * Limits: Cin*Tin*4 < 2^31 bytes per clip. */
int bc_conv1d_select_cfg(int Cout, int Cin, int K, int stride, int dilation, int mode);
/* bc_conv1d_select_cfg_n: the same choice for a launch of B clips with Tout output columns each: a stride-1
 *   multi-tap conv with Tout <= 128 (a streaming chunk, a small batch) may take a narrower tile than the shape
 *   table's (ABI 15; x6 / bf16 results are the same on either tile, h3 agrees to fp32 rounding).  The packed
 *   weights must be packed for the returned cfg. */
int bc_conv1d_select_cfg_n(int Cout, int Cin, int K, int stride, int dilation, int mode, int B, int Tout);
long long bc_conv1d_packed_floats(int Cout, int Cin, int K, int cfg);
int bc_conv1d_pack(const float* w_host, float* packed_host, int Cout, int Cin, int K, int cfg);
int bc_conv1d_fwd(const float* x, const float* w_packed, const float* bias, const float* residual,
                  const float* out_snake_alpha_exp, const float* out_snake_inv_beta,
                  float* y, float* y2, int B, int Cin, int Tin, int Cout, int Tout,
                  int K, int stride, int dilation, int pad_left, int epilogue, int cfg,
                  void* stream);

/* ---- ResidualUnit in one launch (modes 1 "x6", 2 bf16 and 3 "h3"; C in {16, 32, 48, 64, 96}) -------
 * Replaces ResidualUnit.forward (vq/module.py:88-89) after its first Activation1d:
 *   v = x_raw + conv1(snake_mid(conv7_d(x_act)))      (x_act = snake1(x_raw), from the producer)
 *   y = v, or snake_out(v), or y = v and y2 = snake_out(v)  (epilogue as bc_conv1d_fwd)
 * x_raw, x_act, y, y2: [B][C][T]; the k=7 conv keeps length T (pad_left = 3*dilation non-causal,
 * 6*dilation causal; the rest on the right).  w7_packed / w1_packed = bc_conv1d_pack(folded weight,
 * K = 7 / 1, cfg) with cfg = bc_resunit_select_cfg(C, dilation, mode); that returns -1 where the
 * unit does not fit one workgroup, or mode is 0 (then run the two bc_conv1d_fwd calls).  Another
 * candidate tile of the same mode whose rows cover C is accepted too (same results, A/B timing); any
 * other cfg returns BC_ERR_ARG.  The
 * activated k=7 output stays in LDS (never written to memory).  mid_snake_*: the unit's second
 * Activation1d. */
int bc_resunit_select_cfg(int C, int dilation, int mode);
int bc_resunit_fwd(const float* x_raw, const float* x_act, const float* w7_packed, const float* b7,
                   const float* mid_snake_alpha_exp, const float* mid_snake_inv_beta,
                   const float* w1_packed, const float* b1, const float* out_snake_alpha_exp,
                   const float* out_snake_inv_beta, float* y, float* y2, int B, int C, int T,
                   int dilation, int pad_left, int cfg, void* stream);
/* bc_resunit_fwd_snake_in: the same unit with its FIRST Activation1d applied while the k=7 input is
 *   staged (x_act = snake_in(x_raw) is never materialised: the producer writes only x_raw). */
int bc_resunit_fwd_snake_in(const float* x_raw, const float* in_snake_alpha_exp, const float* in_snake_inv_beta,
                            const float* w7_packed, const float* b7, const float* mid_snake_alpha_exp,
                            const float* mid_snake_inv_beta, const float* w1_packed, const float* b1,
                            const float* out_snake_alpha_exp, const float* out_snake_inv_beta, float* y, float* y2,
                            int B, int C, int T, int dilation, int pad_left, int cfg, void* stream);

/* ---- ConvTranspose1d (weight-normed, fused next-Snake epilogue) -------------------------------
 * Replaces: weight_norm(nn.ConvTranspose1d) (vq/module.py:67-72) and CausalConvTranspose1d
 * (vq/module.py:50-57, crop of the last `stride` samples) inside DecoderBlock (vq/module.py:
 * 115-141) (DecoderBlock uses K = 2*stride).  Run as `stride` polyphase convolutions with
 * Kp = bc_convT1d_phase_taps(K, stride) = ceil(K/stride) taps: phase r has
 * W_r[co][ci][j'] = W[ci][co][r + stride*(Kp-1-j')] (0 where that tap index >= K), packed with
 * bc_conv1d_pack(..., K=Kp, cfg), cfg = bc_conv1d_select_cfg(Cout, Cin, Kp, 1, 1, mode).  w_phases is
 * a HOST array of `stride` device pointers.  Output length Tout = (Tin-1)*stride - 2*padding + K +
 * output_padding (the caller passes Tout, which carries output_padding); DecoderBlock non-causal:
 * padding = stride/2 + stride%2, output_padding = stride%2.  Causal (crop of the last `stride`
 * samples): padding = 0, Tout = (Tin-1)*stride + K - stride.  Epilogue as bc_conv1d_fwd. */
int bc_convT1d_phase_taps(int K, int stride);
int bc_convT1d_fwd(const float* x, const float* const* w_phases, const float* bias,
                   const float* out_snake_alpha_exp, const float* out_snake_inv_beta, float* y,
                   float* y2, int B, int Cin, int Tin, int Cout, int Tout, int K, int stride,
                   int padding, int cfg, void* stream);
/* bc_convT1d_fwd_ws (ABI 11): the same transposed convolution and the same values bit for bit, with a
 * workspace of bc_convT1d_workspace_floats(B, Cout, Tout, K, stride, padding, dual) device floats
 * (dual = y2 != NULL): each phase writes its outputs contiguously (16-byte stores) into the workspace
 * and one interleave pass writes y (and y2) in order.  bc_convT1d_fwd writes every phase straight into
 * y with stride-`stride` scalar stores (each output line written in `stride` partial passes); the
 * decoder's stride-5 upsampler ran 2x slower that way.  workspace NULL: as
 * bc_convT1d_fwd. */
long long bc_convT1d_workspace_floats(int B, int Cout, int Tout, int K, int stride, int padding, int dual);
int bc_convT1d_fwd_ws(const float* x, const float* const* w_phases, const float* bias,
                      const float* out_snake_alpha_exp, const float* out_snake_inv_beta, float* y,
                      float* y2, int B, int Cin, int Tin, int Cout, int Tout, int K, int stride,
                      int padding, int cfg, float* workspace, void* stream);

/* ---- SnakeBeta / anti-aliased Activation1d -------------------------------------------------------
 * bc_snake_fwd replaces SnakeBeta.forward (vq/activations.py:107-118).
 * bc_aa_snake_fwd replaces Activation1d.forward with antialias=True (vq/alias_free_torch/act.py:
 * 25-32): UpSample1d (resample.py:25-33) -> SnakeBeta -> DownSample1d (resample.py:47-49,
 * filter.py:86-95).  up_filter / down_filter: the 12-tap buffers `upsample.filter` and
 * `downsample.lowpass.filter` (device, 12 floats each). */
int bc_snake_fwd(const float* x, const float* snake_alpha_exp, const float* snake_inv_beta,
                 float* y, int B, int C, long long T, void* stream);
int bc_aa_snake_fwd(const float* x, const float* snake_alpha_exp, const float* snake_inv_beta,
                    const float* up_filter, const float* down_filter, float* y,
                    int B, int C, int T, void* stream);
/* bc_aa_snake_fwd_ex: the same for Activation1d(up_ratio, down_ratio, up_kernel_size, down_kernel_size)
 * (act.py:8-23; resample.py:10-33 geometry for any ratio): up_filter has up_taps floats, down_filter
 * down_taps; ratios 1..16, taps up to 256 (up_taps >= up_ratio), else 3.  y: [B][C][Tout] with
 * Tout = bc_aa_snake_out_len(T, up_ratio, down_ratio, down_taps) (= T when the ratios are equal and
 * down_taps is even).  (2, 12, 2, 12) runs bc_aa_snake_fwd's kernel. */
long long bc_aa_snake_out_len(int T, int up_ratio, int down_ratio, int down_taps);
int bc_aa_snake_fwd_ex(const float* x, const float* snake_alpha_exp, const float* snake_inv_beta,
                       const float* up_filter, const float* down_filter, float* y, int B, int C, int T, int up_ratio,
                       int up_taps, int down_ratio, int down_taps, void* stream);

/* Diagnostics (bench.py's roofline attribution, no compute): the kernel symbol a bc_conv1d_fwd launch with
 * this cfg (K = the conv's kernel size, before any phase decomposition) or a bc_resunit_fwd launch runs, as
 * rocprofv3 prints it without "void bc::" and the argument list; decided by the launchers' own code.
 * Returns the name's length (written NUL-terminated, truncated to buflen), or -1 for an invalid cfg. */
int bc_conv1d_kernel_name(int cfg, int K, int stride, int dilation, char* buf, int buflen);
int bc_resunit_kernel_name(int cfg, int C, int dilation, char* buf, int buflen);

/* bc_tanh_fwd: nn.Tanh (vq/codec_decoder.py:80) called on its own (decoder.model used as the
 * reference's nn.Sequential); the fused decoder runs it in the last conv's epilogue (epilogue = 1). */
int bc_tanh_fwd(const float* x, float* y, long long n, void* stream);

/* ---- ResLSTM ----------------------------------------------------------------------------------------
 * Replaces ResLSTM.forward (vq/module.py:156-167): rearrange b f t -> b t f, nn.LSTM(H, H,
 * num_layers, batch_first=True) (unidirectional), + skip, rearrange back.  x, out: [B][H][T].
 * Per layer l: w_ih_packed[l] = bc_conv1d_pack(weight_ih_l{l} as [4H][H][1], cfg =
 * bc_conv1d_select_cfg(4H, H, 1, 1, 1, mode)); bias[l] = bias_ih_l{l} + bias_hh_l{l} ([4H], device);
 * w_hh_packed[l] = bc_lstm_pack_hh(weight_hh_l{l}, mode) (same mode as the forward call).  The three
 * pointer arrays are HOST arrays of device pointers.  out = snake(y + x) when out_snake_alpha_exp !=
 * NULL (the Activation1d that follows the ResLSTM in both stacks), else y + x.  workspace:
 * bc_lstm_workspace_floats(B, H, T) device floats.  H % 16 == 0.
 * Modes 1, 2 (= 3) and 3 with H in {256, 512, 1024, 1536}: the recurrence runs as ONE persistent launch per
 * layer (H/8 workgroups that must all be resident at once — checked against the kernel's occupancy,
 * else 3 — W_hh register-resident; mode 1 3xbf16-split, mode 3 2xfp16-split MFMA); otherwise one
 * launch per step (fp32 MFMA).
 * TIMEOUT STATUS: the call zeroes ((int*)workspace)[0] on the stream, and every persistent
 * workgroup that gives up waiting for a neighbour (bounded spin; never in a correct run) adds 1 to it
 * and leaves, so `out` is then WRONG.  The caller must read that int after the call completes and
 * treat nonzero as an error before consuming `out` (the Python package raises BigCodecLibraryError).
 * bc_lstm_status(reset) returns the same count summed over the process's calls (diagnostic),
 * synchronising the device. */
long long bc_lstm_hh_packed_floats(int H, int mode);
int bc_lstm_pack_hh(const float* w_hh_host, float* packed_host, int H, int mode);
long long bc_lstm_workspace_floats(int B, int H, int T);
int bc_lstm_status(int reset);

/* Diagnostic (not on the codec path; bench.py's roofline): nwg workgroups of 4 waves, each wave
 * issuing 16 * iters v_mfma_f32_16x16x32_bf16 on random register operands (16384 FLOP each); out:
 * nwg * 4 device floats.  Timed by the caller, it gives the dense-BF16 rate the device sustains
 * under its clock management, the practical ceiling beside the spec peak. */
int bc_mfma_probe(float* out, int nwg, int iters, void* stream);
int bc_reslstm_fwd(const float* x, float* out, int B, int H, int T, int num_layers,
                   const float* const* w_ih_packed, const float* const* bias,
                   const float* const* w_hh_packed, const float* out_snake_alpha_exp,
                   const float* out_snake_inv_beta, float* workspace, int mode, void* stream);
/* bc_reslstm_fwd_state: bc_reslstm_fwd with carried state for streaming (nn.LSTM's (h0, c0) in, (h_n, c_n)
 *   out): h0 / c0 / hT / cT are [num_layers][H][B] device buffers (unit-major; NULL h0 and c0 = zero
 *   state, NULL hT and cT = not returned).  Runs on the persistent kernel only (modes 1 and 3, H a
 *   multiple of 128 up to 1536); other shapes return 3. */
int bc_reslstm_fwd_state(const float* x, float* out, int B, int H, int T, int num_layers,
                         const float* const* w_ih_packed, const float* const* bias,
                         const float* const* w_hh_packed, const float* out_snake_alpha_exp,
                         const float* out_snake_inv_beta, float* workspace, int mode, const float* h0,
                         const float* c0, float* hT, float* cT, void* stream);

/* bc_reslstm_bidir_fwd: ResLSTM(dimension = D, bidirectional=True) (vq/module.py:150-152: nn.LSTM(D, D / 2,
 *   num_layers, batch_first=True, bidirectional=True)), + skip.  x, out: [B][D][T], H = D / 2, D % 32 == 0.
 *   The pointer arrays hold TWO entries per layer, [2l] = forward and [2l + 1] = backward direction
 *   (torch's weight_ih_l{l} / weight_ih_l{l}_reverse ...), each packed as above but with Cin = D:
 *   w_ih_packed = bc_conv1d_pack(weight_ih as [4H][D][1], cfg = bc_conv1d_select_cfg(4H, D, 1, 1, 1, mode)),
 *   w_hh_packed = bc_lstm_pack_hh(weight_hh, H, mode).  Layer outputs are [forward h | backward h]
 *   (torch's concatenation order); the backward direction runs the forward recurrence over the
 *   time-reversed sequence.  workspace: bc_reslstm_bidir_workspace_floats(B, D, T) floats, same timeout
 *   status contract as bc_reslstm_fwd.  No carried state (streaming models are unidirectional). */
long long bc_reslstm_bidir_workspace_floats(int B, int D, int T);
int bc_reslstm_bidir_fwd(const float* x, float* out, int B, int D, int T, int num_layers,
                         const float* const* w_ih_packed, const float* const* bias,
                         const float* const* w_hh_packed, const float* out_snake_alpha_exp,
                         const float* out_snake_inv_beta, float* workspace, int mode, void* stream);

/* ---- Factorized VQ (codebook_dim == 8) ---------------------------------------------------------
 * bc_vq_prepare_codebook: F.normalize(codebook) and its row sums of squares
 *   (vq/factorized_vector_quantize.py:99,105).
 * bc_vq_fwd: FactorizedVectorQuantize.forward in eval mode (factorized_vector_quantize.py:29-76):
 *   z [B][D][T] -> in_proj (folded WN Linear, w_in [8][D], b_in [8]) -> decode_latents (:93-108) ->
 *   idx [B][T] int64; z_e_out [B][8][T] (optional, may be NULL); post_out [B][D][T] = out_proj of
 *   the straight-through z_q (optional, may be NULL; w_out [D][8], b_out [D]).
 * bc_vq_argmin: decode_latents' search alone: z_e rows [N][8] -> idx [N] int64.  Given the same
 *   z_e the indices equal the reference's ("VQ exactness").
 * bc_vq2emb: FactorizedVectorQuantize.vq2emb (:78-81): idx[n*idx_stride] -> emb [N][D] (= (B,T,D)
 *   as the reference returns); w_out == NULL means proj=False (emb = codebook rows, D == dim);
 *   accumulate != 0 adds into emb (ResidualVQ.vq2emb sum, residual_vq.py:42-48).
 * bc_rvq_update: ResidualVQ bookkeeping (residual_vq.py:31-33): residual -= q; out (+)= q. */
int bc_vq_prepare_codebook(const float* codebook, float* codebook_norm, float* codebook_sq,
                           int n_codes, int dim, void* stream);
int bc_vq_fwd(const float* z, const float* w_in, const float* b_in, const float* codebook,
              const float* codebook_norm, const float* codebook_sq, const float* w_out,
              const float* b_out, long long* idx, float* z_e_out, float* post_out,
              int B, int D, int T, int n_codes, int dim, void* stream);
int bc_vq_argmin(const float* z_e, const float* codebook_norm, const float* codebook_sq,
                 long long* idx, long long N, int n_codes, int dim, void* stream);
int bc_vq2emb(const long long* idx, long long idx_stride, const float* codebook,
              const float* w_out, const float* b_out, float* emb, long long N, int D, int n_codes,
              int dim, int accumulate, void* stream);
int bc_rvq_update(float* residual, float* out, const float* q, long long n, int first,
                  void* stream);
/* bc_vq2emb_ct: the token -> audio entry (codec_decoder.py:96-99 vq2emb, then the caller's
 *   transpose(1, 2) before decoder(x, vq=False)): idx[B][T][nq] int64 -> emb[B][D][T], summed over the
 *   nq quantizers in the reference's order.  Quantizer parameters stacked: codebooks [nq][n_codes][dim],
 *   w_out [nq][D][dim] (folded weight norm), b_out [nq][D].  1 <= nq <= 8, dim == 8.  An index outside
 *   [0, n_codes) gives NaN in its column (never an out-of-range read). */
int bc_vq2emb_ct(const long long* idx, int nq, const float* codebooks, const float* w_out,
                 const float* b_out, float* emb, int B, int T, int D, int n_codes, int dim, void* stream);

/* bc_fsq_fwd: FSQ.forward (vendored lucidrains finite_scalar_quantization.py:205-262; the decoder's
 *   fsq=True quantizer, codec_decoder.py:41-47, 85-92), eval, channel_first: z[B][D][T] ->
 *   idx[B][T] int32 and (optional) post[B][D][T] = project_out(codes).  w_in [d][D], b_in [d], w_out [D][d],
 *   b_out [D]; consts[5][d] = half_l, offset, shift, half_width, basis (float32, from the reference's own
 *   expressions); 1 <= d <= 8. */
int bc_fsq_fwd(const float* z, const float* w_in, const float* b_in, const float* w_out, const float* b_out,
               const float* consts, int* idx, float* post, int B, int D, int T, int d, void* stream);

/* bc_fsq_codes: FSQ.indices_to_codes (finite_scalar_quantization.py:159-192), channel_first, one codebook: the
 *   fsq=True decoder's token -> latent step (its vq2emb raises AttributeError in the reference: FSQ has no vq2emb,
 *   codec_decoder.py:96-99).  idx[B][T] (idx_bits 32: int32, 64: int64) -> post[B][D][T] = project_out(codes),
 *   codes[j] = ((idx // basis[j]) % levels[j] - levels[j] // 2) / (levels[j] // 2) with torch's floor // and %
 *   (any integer maps to a grid point, as in the reference), basis = cumprod([1] + levels[:-1]).  levels is a
 *   HOST array of d ints >= 2; w_out [D][d], b_out [D] as in bc_fsq_fwd, whose post it reproduces bit for bit
 *   for the indices it returned.  1 <= d <= 8. */
int bc_fsq_codes(const void* idx, int idx_bits, const int* levels, const float* w_out, const float* b_out,
                 float* post, int B, int D, int T, int d, void* stream);

/* bc_stream_window: one step of a causal stream's carried state (audiotokenization_amd/streaming.py; the reference has
 *   no streaming mode, its whole-sequence causal convs, vq/module.py:11-48, define the result): for each row (b, c)
 *   win[b][c][j] = j < P ? ctx[b][c][j] : act(x[b][c][j - P]) for j < P + n, and ctx_out[b][c][i] = win[b][c][n + i]
 *   for i < P.  act = SnakeBeta with (snake_alpha_exp, snake_inv_beta) as bc_snake_fwd takes them, or the identity
 *   when both are NULL; ctx NULL reads zeros (a stream's start).  x is read at x + b * x_batch_stride + c *
 *   x_row_stride + t (floats), so a strided view works; win is [B][C][P + n], ctx / ctx_out [B][C][P] (ctx_out may be
 *   NULL only when P == 0) and must not overlap ctx. */
int bc_stream_window(const float* x, long long x_batch_stride, long long x_row_stride, const float* ctx,
                     const float* snake_alpha_exp, const float* snake_inv_beta, float* win, float* ctx_out, int B, int C,
                     int n, int P, void* stream);

/* ---- Real-audio ingest ------------------------------------------------------------------------
 * bc_resample_sinc: torchaudio.transforms.Resample(orig, new) as extract_indices.py:129-132 and
 *   data_module.py:95-98 call it: x[B][Lin] -> y[b * y_pitch + o], o < Lout = ceil(new * Lin / orig)
 *   (y_pitch >= Lout leaves room for extract_indices.py:135-137's pad_to_stride zeros), with
 *   orig / new already divided by their gcd and kern[new][taps] the host-built sinc-Hann filters
 *   (audiotokenization_amd/ingest.py sinc_resample_kernel, taps = 2 * width + orig). */
int bc_resample_sinc(const float* x, float* y, const float* kern, int B, long long Lin, long long Lout,
                     long long y_pitch, int orig, int new_freq, int taps, int width, void* stream);

/* ---- FLAC decoding (host code, no device memory) -----------------------------------------------
 * Replaces soundfile's read of the reference's LibriTTS / LibriSpeech .flac utterances
 * (extract_indices.py:98-106: sf.SoundFile(...).read(dtype='float32', always_2d=True)).  RFC 9639 streams:
 * all subframe types, Rice / escaped residuals, wasted bits, stereo decorrelations, 4-32 bit samples.
 * bc_flac_info: STREAMINFO of an in-memory stream (total_samples 0 = unknown); returns 0, 1 (bad argument),
 *   2 (not FLAC / corrupt), 3 (unsupported).
 * bc_flac_decode: every frame into out[channel * max_samples + i] (HOST memory), int32 when out_int32 != 0,
 *   else float32 = sample * 2^-(bits - 1) (libsndfile's normalised float read); check_crc verifies the
 *   frame-header CRC-8 and frame CRC-16.  Returns samples per channel, or -1 bad argument, -2 corrupt,
 *   -3 unsupported, -4 CRC mismatch, -5 more than max_samples samples. */
int bc_flac_info(const unsigned char* data, long long n, int* sample_rate, int* channels, int* bits,
                 long long* total_samples);
long long bc_flac_decode(const unsigned char* data, long long n, void* out, int out_int32, long long max_samples,
                         int check_crc);

/* ---- Layout helpers & synthetic input --------------------------------------------------------
 * bc_btc_to_ctb: x[B][C][T] -> y[C][T][B];  bc_ctb_to_btc_add: out = transpose(y) + skip.
 * bc_synth_clips: x[B][T] white noise, clip i = clip0 + b (SURVEY.md §8(d) spec). */
int bc_btc_to_ctb(const float* x, float* y, int B, int C, int T, void* stream);
int bc_ctb_to_btc_add(const float* y, const float* skip, float* out, int B, int C, int T,
                      void* stream);
int bc_synth_clips(float* x, int B, long long T, long long clip0, void* stream);

/* ---- Bounds-checked debug build (no reference counterpart: SURVEY.md §5 row 2) ------------------------------
 * libbigcodec_hip.so built with -DBC_DEBUG (build_lib.build(debug=True) -> audiotokenization_amd/_debug/, loaded by
 * the Python package when BIGCODEC_DEBUG=1) checks the indices of the kernels' computed global accesses (conv /
 * ResidualUnit epilogue stores and residual reads, weight copies, ResLSTM output stores); a failed check is counted
 * and its access skipped, so a bad launch reports instead of faulting the GPU.
 * bc_debug_status(out[2]): out[0] = failed checks since the last call, out[1] = the first failing source line
 *   (0 = none); reads and clears; synchronises the device.  Returns 3 (unsupported) in the product build.
 * bc_debug_selftest(n, stream): a kernel whose n lanes fail one check each on purpose, touching no memory
 *   outside the debug words (the mechanism's own test).  Returns 3 in the product build. */
int bc_debug_status(unsigned int* out);
int bc_debug_selftest(int n, void* stream);

/* ---- Launch timer of the composite calls (ABI 17; no reference counterpart: the measurement row SURVEY.md §8(d)) --
 * The Python layer times every conv / ResidualUnit launch it makes itself; the kernels that bc_reslstm_fwd[_state],
 * bc_reslstm_bidir_fwd and bc_vq_fwd launch inside one call (the layout transposes, the ResLSTM input projection and
 * its pre-split planes, the persistent recurrence, the VQ) are only visible to the library.  While enabled, each of
 * those launches is bracketed by HIP events recorded on the stream it is launched on.
 * bc_launch_timer_enable(on): 1 starts a fresh recording (stale records are dropped), 0 stops it (records kept).
 * bc_launch_timer_read(max, names, ms, flops, bytes): with max <= 0 or a null array, returns the number of records
 *   and keeps them; otherwise synchronises the recorded events, copies the first max records (names: max x 64 bytes,
 *   NUL-terminated kernel symbols; ms: event-timed duration; flops / bytes: the launch's algorithmic work), clears
 *   all of them and returns their number (-1 on a HIP error). */
int bc_launch_timer_enable(int on);
int bc_launch_timer_read(int max, char* names, float* ms, double* flops, double* bytes);

#ifdef __cplusplus
}
#endif
#endif /* BIGCODEC_H */
