"""Causal streaming encode (audiotokenization_amd/streaming.py) on the MI355X.

Property (size-independent, the reference has no streaming mode of its own): for a causal encoder the
concatenated latents of a chunked stream equal the whole-sequence encode of the concatenated audio.
  x6 precision (exact operand splits, tile-independent): two different chunkings and the whole-sequence pass
    agree BIT FOR BIT (round 4: the stream runs the same one-launch ResidualUnits over its context windows and
    the same Snake epilogues as the whole pass; measured 0.00e+00 in h3 too at these sizes);
  h3 precision (per-tile block scales): <= 1e-5;
  VQ indices of stream and whole pass equal except certified near-ties (test_gpu_model.py's rule);
and the whole-sequence causal encoder itself is checked against the CPU oracle on the same audio.
"""
import pytest
import torch

from audiotokenization_amd import _lib as L
from audiotokenization_amd import synth
from audiotokenization_amd.streaming import StreamingEncoder
from helpers import assert_close_rel, build_models, index_mismatches, max_rel_err, top2_gap, torch_sd
from oracle import bigcodec_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model,B,chunks", [("base", 2, (1000, 3000)), ("debug", 2, (960, 1920)),
                                            ("default", 1, (1200, 2400)), ("default", 1, (200, 600))])
@pytest.mark.parametrize("sprec", ["x6", "h3"])
def test_stream_equals_whole_sequence(dev, model, B, chunks, sprec):
    old = L.precision_mode()
    try:
        L.set_precision(sprec)
        enc, dec, esd, dsd, ek, _ = build_models(model, device=dev, causal=True)
        n = 6000 if model != "debug" else 5760
        x = torch.from_numpy(synth.synth_clips(B, n, clip0=11)).unsqueeze(1).to(dev)
        s = StreamingEncoder(enc)
        with torch.no_grad():
            full = enc(x)
            a = s.encode(x, chunks[0])
            b = s.encode(x, chunks[1])
            torch.cuda.synchronize()
        assert a.shape == full.shape == b.shape
        if sprec == "x6":
            assert torch.equal(a, b), f"two chunkings differ: {max_rel_err(a, b):.3e}"
            assert torch.equal(a, full), f"stream != whole pass: {max_rel_err(a, full):.3e}"
        err = max_rel_err(a, full)
        print(f"stream {model} [{sprec}] chunks {chunks}: max rel diff to the whole pass {err:.2e}, "
              f"chunkings {max_rel_err(a, b):.2e}")
        assert err <= (1e-6 if sprec == "x6" else 1e-5), err
        with torch.no_grad():
            c_full = dec(full, vq=True)[1].cpu()
            c_a = dec(a, vq=True)[1].cpu()
            lat_ref = O.encoder_forward(x.cpu(), torch_sd(esd), ek)
            _, _, _, ze = O.fvq_forward(lat_ref, torch_sd(dsd), "quantizer.layers.0.", return_ze=True)
        gap = top2_gap(ze, torch.from_numpy(dsd["quantizer.layers.0._codebook.weight"]))
        index_mismatches(c_a.numpy(), c_full.numpy(), gap)
        assert_close_rel(full.cpu(), lat_ref, 1e-4, "causal whole-sequence latent vs oracle")
    finally:
        L._mode = old


def test_stream_rejects_bad_chunks_and_non_causal(dev):
    enc, *_ = build_models("debug", device=dev, causal=True)
    s = StreamingEncoder(enc)
    with pytest.raises(ValueError):
        s.push(torch.zeros(1, 1, 321, device=dev))
    enc_nc, *_ = build_models("debug", device=dev)
    with pytest.raises(ValueError):
        StreamingEncoder(enc_nc)


@pytest.mark.parametrize("model,B,chunks", [("base", 2, (7, 16)), ("debug", 2, (5, 12)), ("default", 1, (6, 13))])
@pytest.mark.parametrize("sprec", ["x6", "h3"])
def test_stream_decode_equals_whole_sequence(dev, model, B, chunks, sprec):
    """Causal streaming DECODE (streaming.StreamingDecoder; vq/module.py:50-57 CausalConvTranspose1d carried as one
    input frame per upsampler): the chunked stream of post-VQ latents equals the whole-sequence causal decode,
    two chunkings and the whole pass bit for bit in x6, <= 1e-5 of max|wav| in h3; the token stream (vq2emb per
    chunk) equals the whole token decode the same way; the whole-sequence causal decoder is within 1e-4 of the oracle."""
    from audiotokenization_amd.streaming import StreamingDecoder

    old = L.precision_mode()
    try:
        L.set_precision(sprec)
        enc, dec, esd, dsd, ek, dk = build_models(model, device=dev, causal=True)
        n = 6000 if model != "debug" else 5760
        x = torch.from_numpy(synth.synth_clips(B, n, clip0=23)).unsqueeze(1).to(dev)
        s = StreamingDecoder(dec)
        with torch.no_grad():
            post, codes, _ = dec(enc(x), vq=True)
            full = dec(post, vq=False)
            a = s.decode(post, chunks[0])
            b = s.decode(post, chunks[1])
            tok = codes.permute(1, 2, 0).contiguous()  # (B, F, Nq): the token files' layout, batched
            s.reset()
            t = torch.cat([s.tokens(tok[:, i:i + chunks[0]]) for i in range(0, tok.shape[1], chunks[0])], dim=2)
            # (the VQ forward's post embedding is straight-through, z_e + (z_q - z_e): the token path decodes z_q)
            full_tok = dec(dec.quantizer.vq2emb_ct(tok), vq=False)
            torch.cuda.synchronize()
        assert a.shape == full.shape == b.shape == (B, 1, n)
        if sprec == "x6":
            assert torch.equal(a, b), f"two chunkings differ: {max_rel_err(a, b):.3e}"
            assert torch.equal(a, full) and torch.equal(t, full_tok), "x6 stream decode != whole pass"
        err = max_rel_err(a, full)
        print(f"stream decode {model} [{sprec}] chunks {chunks}: max rel diff to the whole pass {err:.2e}, "
              f"chunkings {max_rel_err(a, b):.2e}, token stream vs whole token decode {max_rel_err(t, full_tok):.2e}")
        assert err <= (1e-6 if sprec == "x6" else 1e-5), err
        assert max_rel_err(t, full_tok) <= (1e-6 if sprec == "x6" else 1e-5)
        wav_ref = O.decoder_forward(post.cpu(), torch_sd(dsd), dk)
        assert_close_rel(full.cpu(), wav_ref, 1e-4, "causal whole-sequence decode vs oracle")
    finally:
        L._mode = old


def test_stream_decode_rejects_non_causal(dev):
    from audiotokenization_amd.streaming import StreamingDecoder

    _, dec, *_ = build_models("debug", device=dev)
    with pytest.raises(ValueError):
        StreamingDecoder(dec)


@pytest.mark.parametrize("P,n,strided,act,first", [(18, 100, False, True, False), (54, 20, True, True, False),
                                                   (6, 37, True, False, True), (0, 9, True, False, True),
                                                   (3, 3, False, True, True)])
def test_stream_window_kernel(dev, P, n, strided, act, first):
    """bc_stream_window (the stream's carried state): win = [ctx | act(x)], ctx_out = win[..., -P:], bit for bit
    against the product's own Snake op and plain copies; strided chunk views (a ResidualUnit's output columns
    [P:] of its window), P > n (the context outlives a short chunk), a missing context = zeros."""
    from audiotokenization_amd import ops

    ns = ops.load()
    g = torch.Generator().manual_seed(P * 131 + n)
    B, C = 3, 40
    base = torch.randn(B, C, n + 11, generator=g).to(dev)
    x = base[:, :, 11:] if strided else base[:, :, :n].contiguous()
    ctx = None if first else torch.randn(B, C, P, generator=g).to(dev)
    a = torch.rand(C, generator=g).add(0.5).to(dev) if act else None
    ib = torch.rand(C, generator=g).add(0.5).to(dev) if act else None
    win, nctx = ns.stream_window(x, ctx, a, ib, P)
    xa = ns.snake(x.contiguous(), a, ib) if act else x
    ref = torch.cat([ctx if ctx is not None else torch.zeros(B, C, P, device=dev), xa], dim=2)
    assert torch.equal(win, ref)
    assert nctx.shape == (B, C, P) and torch.equal(nctx, ref[:, :, ref.shape[2] - P:])


@pytest.mark.parametrize("sprec", ["h3", "x6"])
def test_stream_graph_equals_eager_stream(dev, sprec):
    """StreamGraph (one HIP-graph replay per chunk): the encode and decode streams equal the eager streams bit for
    bit, when captured on a fresh stream and when captured mid-stream (the graph takes the eager stream's carried
    context and ResLSTM state over); a chunk of another shape is refused; the ResLSTM status words are read."""
    from audiotokenization_amd.streaming import StreamingDecoder

    old = L.precision_mode()
    try:
        L.set_precision(sprec)
        enc, dec, *_ = build_models("default", device=dev, causal=True)
        B, n, ch = 2, 6000, 1200
        x = torch.from_numpy(synth.synth_clips(B, n, clip0=31)).unsqueeze(1).to(dev)
        with torch.no_grad():
            eager = StreamingEncoder(enc).encode(x, ch)
            s = StreamingEncoder(enc)
            g = s.graph(x[..., :ch])
            fresh = torch.cat([g.push(x[..., i:i + ch]).clone() for i in range(0, n, ch)], dim=2)
            s2 = StreamingEncoder(enc)
            first = s2.push(x[..., :ch])  # eager, then the graph continues the same stream
            g2 = s2.graph(x[..., :ch])
            mid = torch.cat([first] + [g2.push(x[..., i:i + ch]).clone() for i in range(ch, n, ch)], dim=2)
            with pytest.raises(ValueError):
                g2.push(x[..., :ch // 2])
            post = dec(eager, vq=True)[0]
            fc = 6
            d_eager = StreamingDecoder(dec).decode(post, fc)
            sd = StreamingDecoder(dec)
            gd = sd.graph(post[..., :fc])
            d_graph = torch.cat([gd.push(post[..., i:i + fc]).clone() for i in range(0, post.shape[-1], fc)], dim=2)
            torch.cuda.synchronize()
        assert torch.equal(fresh, eager), f"graph stream != eager stream: {max_rel_err(fresh, eager):.3e}"
        assert torch.equal(mid, eager), f"mid-stream graph != eager stream: {max_rel_err(mid, eager):.3e}"
        assert torch.equal(d_graph, d_eager), f"graph decode stream != eager: {max_rel_err(d_graph, d_eager):.3e}"
        assert s.samples == n and sd.samples == post.shape[-1] * dec.hop_length
        assert g._status, "the graph holds the ResLSTM status words"
        g.check()
    finally:
        L._mode = old


def test_stream_bf16_equals_whole_pass(dev):
    """bf16 conv products (config 5's arithmetic) in the stream: one bf16 plane per operand, no block scales, so the
    products do not depend on the tiling and the encode / decode streams equal the bf16 whole-sequence pass bit for
    bit, like x6 (the fidelity of bf16 itself is test_gpu_configs.py's concern)."""
    from audiotokenization_amd.streaming import StreamingDecoder

    old = L.precision_mode()
    try:
        L.set_precision("bf16")
        enc, dec, *_ = build_models("default", device=dev, causal=True)
        x = torch.from_numpy(synth.synth_clips(2, 6000, clip0=41)).unsqueeze(1).to(dev)
        with torch.no_grad():
            full = enc(x)
            a = StreamingEncoder(enc).encode(x, 1200)
            post = dec(full, vq=True)[0]
            wav = dec(post, vq=False)
            w = StreamingDecoder(dec).decode(post, 7)
            torch.cuda.synchronize()
    finally:
        L._mode = old
    print(f"bf16 stream: encode {max_rel_err(a, full):.2e}, decode {max_rel_err(w, wav):.2e} vs the whole pass")
    assert torch.equal(a, full) and torch.equal(w, wav)
