"""Model-level parity on the MI355X against the reference's golden outputs (tests/golden/) and
size-independent properties at BASELINE.json's full sizes.

Tolerances (fp32 throughout, north_star "reconstructed waveforms within a stated fp32 tolerance"):
  latent (encoder output)      max|d| / max|ref| <= 1e-4
  VQ indices                   equal, except frames whose fp64 top-2 distance gap < 1e-6 (helpers.GAP_TOL)
                               (reported; a near-tie flips under any fp32 reassociation —
                               SURVEY.md §0 item 7: two valid CPU builds already differ)
  waveform (decoding the reference's own z_q)   MSE <= 1e-12 and max|d| <= 1e-5
"""
import os

import numpy as np
import pytest
import torch

from helpers import assert_close_rel, build_models, index_mismatches, torch_sd
from oracle import bigcodec_oracle as O

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
MODEL_FILES = sorted(f for f in os.listdir(GOLDEN) if f.startswith("model_"))
LAYER_FILES = sorted(f for f in os.listdir(GOLDEN) if f.startswith("layers_"))


@pytest.mark.parametrize("fname", MODEL_FILES)
def test_model_against_reference(dev, golden, fname, prec):
    g = golden(fname)
    meta = g["meta"]
    enc, dec, _, _, ek, dk = build_models(meta["model"], device=dev, **meta["overrides"])
    x = torch.from_numpy(g["x"]).to(dev)
    with torch.no_grad():
        lat = enc(x)
        post, codes, loss = dec(lat, vq=True)
        torch.cuda.synchronize()
    assert_close_rel(lat.cpu(), torch.from_numpy(g["latent"]), 1e-4, "latent")
    n_bad, worst = index_mismatches(codes.cpu().numpy(), g["codes"], g["gap"])
    print(f"{fname}: {n_bad} index mismatches (worst certified gap {worst:.2e}) of {codes.numel()}")
    assert codes.shape == g["codes"].shape and codes.dtype == torch.int64
    assert float(loss.abs().sum()) == 0.0
    if "wav" in g:
        # decode the reference's own z_q: isolates the decoder error
        wav = dec(torch.from_numpy(g["post"]).to(dev), vq=False)
        torch.cuda.synchronize()
        w, ref = wav.cpu().double(), torch.from_numpy(g["wav"]).double()
        assert w.shape == ref.shape
        mse = float(((w - ref) ** 2).mean())
        mx = float((w - ref).abs().max())
        print(f"{fname}: decoder mse {mse:.2e} max {mx:.2e}")
        assert mse <= 1e-12 and mx <= 1e-5
        emb = dec.vq2emb(torch.from_numpy(g["codes"]).permute(1, 2, 0).contiguous().to(dev)).cpu()
        assert_close_rel(emb, torch.from_numpy(g["vq2emb"]), 1e-6, "vq2emb")


@pytest.mark.parametrize("fname", LAYER_FILES)
def test_layers_against_reference(dev, golden, fname):
    """Per-stage known answers: feed each encoder/decoder stage the reference's own input."""
    g = golden(fname)
    meta = g["meta"]
    enc, dec, _, _, _, _ = build_models(meta["model"], device=dev, **meta["overrides"])
    prev = g["x"]
    with torch.no_grad():
        for i, m in enumerate(enc.block):  # stand-alone module calls (the final Snake runs unfused here)
            out = m(torch.from_numpy(prev).to(dev))
            assert_close_rel(out.cpu(), torch.from_numpy(g[f"enc_{i}"]), 2e-5, f"enc stage {i}")
            prev = g[f"enc_{i}"]
        # decoder stages up to the last conv (its Snake and the final nn.Tanh are fused in decode())
        post, _, _ = dec(torch.from_numpy(g[f"enc_{meta['n_enc'] - 1}"]).to(dev), vq=True)
        prev = g[f"enc_{meta['n_enc'] - 1}"]
        h = post
        for i in range(meta["n_dec"] - 3):
            h = dec.model[i](h)
            assert_close_rel(h.cpu(), torch.from_numpy(g[f"dec_{i}"]), 1e-4, f"dec stage {i}")
        wav = dec(post, vq=False).cpu()
        assert_close_rel(wav, torch.from_numpy(g[f"dec_{meta['n_dec'] - 1}"]), 1e-4, "decoder out")


def test_bf16_precision_index_mismatch_rate(dev, golden):
    """Config 5's bf16 conv stack is not index-exact (expect a few %); the rate on the
    default-model golden is reported and bounded, and the fp32-accurate path still matches exactly."""
    from audiotokenization_amd import _lib as L

    g = golden("model_default.npz")
    meta = g["meta"]
    enc, dec, *_ = build_models(meta["model"], device=dev, **meta["overrides"])
    x = torch.from_numpy(g["x"]).to(dev)
    old = L.precision_mode()
    try:
        L.set_precision("bf16")
        with torch.no_grad():
            codes = dec(enc(x), vq=True)[1].cpu().numpy()
    finally:
        L._mode = old
    rate = float((codes != g["codes"]).mean())
    print(f"bf16 conv products: index mismatch rate {rate:.4f} over {codes.size} frames")
    # measured 0.042 (5 of 120 frames; 2.9 % over config 5's 115 200): the bound is about twice the config-5 rate
    assert rate < 0.06


def test_lightning_shim_surface(dev, golden):
    """extract_indices.py:353-363 and inference_full.py:557-561 call shapes on the shim."""
    from audiotokenization_amd import CodecLightningModule, preset
    from audiotokenization_amd.extract import BigCodecModel, indices_to_numpy, pad_like_inference_full
    from helpers import synth_load

    g = golden("model_config1_default.npz")
    lm = CodecLightningModule(preset("default"))
    synth_load(lm.encoder, "encoder.")
    synth_load(lm.decoder, "decoder.")
    # strict load of a Lightning-style checkpoint dict carrying training-only keys too
    sd = {**lm.state_dict(), "discriminator.dummy": torch.zeros(1), "spec_discriminator.x": torch.zeros(1)}
    lm.load_state_dict({"state_dict": sd}, strict=True)
    assert "model" not in dict(lm.named_children())
    lm.eval().to(dev)
    x24k = torch.from_numpy(g["x"][..., :24000]).to(dev)
    x = pad_like_inference_full(x24k)  # inference_full.py:712 (+200 on a multiple of 200)
    assert x.shape[-1] == 24200 and torch.equal(x.cpu(), torch.from_numpy(g["x"]))
    out = BigCodecModel(lm, reconstruct=True)(x)
    n_bad, _ = index_mismatches(out["indices"].cpu().numpy(), g["codes"], g["gap"])
    assert out["x_rec"].shape == (1, 1, 24200)
    arr = indices_to_numpy(out["indices"])
    assert arr.dtype == np.int16 and arr.shape == (121, 1)
    codes5 = lm.quantize(lm.encode(x))[1]
    assert torch.equal(codes5, out["indices"])
    wav = lm.inference(x[:, 0])
    assert wav.shape == (1, 24200)


def _full_model(dev, name="default"):
    enc, dec, esd, dsd, ek, dk = build_models(name, device=dev)
    return enc, dec, esd, dsd, ek, dk


@pytest.mark.parametrize("precision", ["h3", "x6"])
def test_full_size_batch_invariance_and_determinism(dev, precision):
    """BASELINE config 2 shape (10 s @24 kHz clips, default model): repeated runs give bitwise identical
    LATENTS (every precision has a fixed accumulation order, so any difference is a race; a code-only check
    misses a drift that moves no index), and a clip's indices do not depend on which batch it is
    encoded in.  The first forward runs after a forward in the other precision, as in the suite's order."""
    from audiotokenization_amd import _lib
    from audiotokenization_amd.extract import synth_batch

    enc, dec, *_ = _full_model(dev)
    old = _lib.precision_mode()
    try:
        with torch.no_grad():
            xb = synth_batch(8, 240000, 0, dev)
            _lib.set_precision("x6" if precision == "h3" else "h3")
            enc(xb)  # leaves the other precision's data in every reused workspace
            _lib.set_precision(precision)
            l1 = enc(xb)
            l2 = enc(xb)
            c1 = dec(l1, vq=True)[1]
            c2 = dec(l2, vq=True)[1]
            cs = torch.cat([dec(enc(xb[i:i + 1]), vq=True)[1] for i in (0, 5)], dim=1)
            torch.cuda.synchronize()
    finally:
        _lib._mode = old
    assert c1.shape == (1, 8, 1200)
    if not torch.equal(l1, l2):
        from helpers import error_profile

        raise AssertionError(f"[{precision}] two forwards of one batch differ: {error_profile(l1, l2)}")
    assert torch.equal(c1, c2)
    assert torch.equal(c1[:, [0, 5]], cs)
    assert len(torch.unique(c1)) > 50


def test_full_size_clip_against_oracle(dev, prec):
    """One full 10 s clip (default model) encoded on the GPU vs the CPU oracle; mismatches only at
    certified near-ties."""
    from audiotokenization_amd import synth

    enc, dec, esd, dsd, ek, dk = _full_model(dev)
    x = torch.from_numpy(synth.synth_clips(1, 240000, clip0=3)).unsqueeze(1)
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    with torch.no_grad():
        lat_ref = O.encoder_forward(x, torch_sd(esd), ek)
        _, codes_ref, _ = O.rvq_forward(lat_ref, torch_sd(dsd))
        _, _, _, ze_ref = O.fvq_forward(lat_ref, torch_sd(dsd), "quantizer.layers.0.", return_ze=True)
        lat = enc(x.to(dev))
        codes = dec(lat, vq=True)[1]
        torch.cuda.synchronize()
    assert_close_rel(lat.cpu(), lat_ref, 1e-4, "latent 10 s")
    from helpers import top2_gap

    gap = top2_gap(ze_ref, torch.from_numpy(dsd["quantizer.layers.0._codebook.weight"]))
    n_bad, worst = index_mismatches(codes.cpu().numpy(), codes_ref.numpy(), gap)
    print(f"10 s default clip [{prec}]: {n_bad} / 1200 index mismatches, worst certified gap {worst:.2e}")


@pytest.mark.parametrize("nq", [2, 4])
def test_rvq_multi_quantizer_against_reference(dev, golden, nq):
    """vq_num_quantizers > 1 against the REFERENCE's ResidualVQ (tests/golden/rvq_base_nq*.npz,
    residual_vq.py:21-40): the reference latent through our RVQ on the GPU -> codes (Nq, B, F) equal,
    except at a frame certified at its first differing layer (the fixture's per-layer fp64 top-2 gap <
    GAP_TOL; later layers then see another residual); post-VQ within 1e-5; vq2emb within 1e-6.  Then
    the whole base encoder + RVQ from the synthetic clip."""
    from audiotokenization_amd import synth
    from helpers import GAP_TOL

    g = golden(f"rvq_base_nq{nq}.npz")
    meta = g["meta"]
    enc, dec, *_ = build_models("base", device=dev, vq_num_quantizers=nq)
    with torch.no_grad():
        post, codes, loss = dec(torch.from_numpy(g["latent"]).to(dev), vq=True)
        x = torch.from_numpy(synth.synth_clips(meta["n_clips"], meta["n_samples"], clip0=meta["clip0"])).unsqueeze(1)
        codes_e2e = dec(enc(x.to(dev)), vq=True)[1]
        emb = dec.vq2emb(torch.from_numpy(g["codes"]).permute(1, 2, 0).contiguous().to(dev))
        torch.cuda.synchronize()
    assert tuple(codes.shape) == g["codes"].shape and float(loss.abs().sum()) == 0.0
    for name, c in (("latent-fed", codes), ("end to end", codes_e2e)):
        gi, wi = c.cpu().numpy().reshape(nq, -1), g["codes"].reshape(nq, -1)
        gap = g["gap"].reshape(nq, -1)
        bad = np.nonzero((gi != wi).any(0))[0]
        for f in bad:
            first = int(np.nonzero(gi[:, f] != wi[:, f])[0][0])
            assert gap[first, f] < GAP_TOL, f"{name}: frame {f} layer {first} flipped at gap {gap[first, f]:.2e}"
        print(f"rvq nq={nq} [{name}]: {bad.size} / {gi.shape[1]} frames differ")
        if name == "latent-fed":
            ok = np.ones(gi.shape[1], bool)
            ok[bad] = False
            gq = post.cpu().permute(0, 2, 1).reshape(-1, post.shape[1])[ok]
            wq = torch.from_numpy(g["post"]).permute(0, 2, 1).reshape(-1, post.shape[1])[ok]
            assert_close_rel(gq, wq, 1e-5, f"rvq nq={nq} post")
    assert_close_rel(emb.cpu(), torch.from_numpy(g["vq2emb"]), 1e-6, f"rvq nq={nq} vq2emb")


def test_bidirectional_rnn_encoder_against_oracle(dev):
    """rnn_bidirectional=True (codec_encoder.py:18,46, a constructor option no shipped config sets): the
    'base' encoder with a bidirectional ResLSTM against the CPU oracle (torch's LSTM inside)."""
    enc, dec, esd, dsd, ek, dk = build_models("base", device=dev, rnn_bidirectional=True)
    assert ek["rnn_bidirectional"]
    from audiotokenization_amd import synth

    x = torch.from_numpy(synth.synth_clips(2, 9600, clip0=11)).unsqueeze(1)
    with torch.no_grad():
        lat_ref = O.encoder_forward(x, torch_sd(esd), ek)
        lat = enc(x.to(dev))
        torch.cuda.synchronize()
    assert_close_rel(lat.cpu(), lat_ref, 1e-4, "bidirectional-rnn latent")
