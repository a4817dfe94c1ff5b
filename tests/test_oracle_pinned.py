"""The CPU oracle (oracle/bigcodec_oracle.py, oracle/vq_oracle.c) reproduces the reference's own
outputs (tests/golden/, produced from /root/reference by tools/make_golden.py) bit for bit."""
import glob
import os

import numpy as np
import pytest
import torch

from helpers import build_models, torch_sd
from oracle import bigcodec_oracle as O
from oracle import vq_c

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
MODEL_FILES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "model_*.npz")))
LAYER_FILES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "layers_*.npz")))


@pytest.mark.parametrize("fname", MODEL_FILES)
def test_model_fixture(golden, fname):
    g = golden(fname)
    meta = g["meta"]
    torch.set_num_threads(8)
    _, _, esd, dsd, ek, dk = build_models(meta["model"], **meta["overrides"])
    esd, dsd = torch_sd(esd), torch_sd(dsd)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        lat = O.encoder_forward(x, esd, ek)
        assert torch.equal(lat, torch.from_numpy(g["latent"]))
        post, codes, losses = O.rvq_forward(lat, dsd, "quantizer.", dk["vq_num_quantizers"])
        assert torch.equal(codes, torch.from_numpy(g["codes"]))
        assert torch.equal(post, torch.from_numpy(g["post"]))
        assert torch.equal(losses, torch.zeros(dk["vq_num_quantizers"]))
        if "wav" in g:
            wav = O.decoder_forward(post, dsd, dk)
            assert torch.equal(wav, torch.from_numpy(g["wav"]))
            emb = O.vq2emb(codes.permute(1, 2, 0), dsd, "quantizer.", dk["vq_num_quantizers"])
            assert torch.equal(emb, torch.from_numpy(g["vq2emb"]))


@pytest.mark.parametrize("fname", LAYER_FILES)
def test_layer_fixture(golden, fname):
    g = golden(fname)
    meta = g["meta"]
    _, _, esd, dsd, ek, dk = build_models(meta["model"], **meta["overrides"])
    esd, dsd = torch_sd(esd), torch_sd(dsd)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        lat = O.encoder_forward(x, esd, ek)
        assert torch.equal(lat, torch.from_numpy(g[f"enc_{meta['n_enc'] - 1}"]))
        post, _, _ = O.rvq_forward(lat, dsd)
        wav = O.decoder_forward(post, dsd, dk)
        assert torch.equal(wav, torch.from_numpy(g[f"dec_{meta['n_dec'] - 1}"]))


def test_aa_fixture(golden):
    from audiotokenization_amd.modules import UpSample1d, DownSample1d

    g = golden("aa_activation.npz")
    # the product's init-time Kaiser-sinc restatement equals the reference buffers
    assert np.array_equal(UpSample1d(2, 12).filter.numpy(), g["up_filter"])
    assert np.array_equal(DownSample1d(2, 12).lowpass.filter.numpy(), g["down_filter"])
    fu, fd = torch.from_numpy(g["up_filter"]), torch.from_numpy(g["down_filter"])
    for T in (1, 5, 37, 600):
        sd = {"act.alpha": torch.from_numpy(g[f"alpha_{T}"]), "act.beta": torch.from_numpy(g[f"beta_{T}"]),
              "upsample.filter": fu, "downsample.lowpass.filter": fd}
        y = O.activation(torch.from_numpy(g[f"x_{T}"]), sd, "", True)
        assert torch.equal(y, torch.from_numpy(g[f"y_{T}"])), T


def test_aa_ratios_fixture(golden):
    """Non-default Activation1d ratios / tap counts (act.py:8-23) against the reference's own outputs
    (tools/make_golden_aa_ratios.py): the product's filter buffers and the oracle restatement."""
    from audiotokenization_amd.modules import DownSample1d, UpSample1d

    g = golden("aa_activation_ratios.npz")
    meta = g["meta"]
    for ci, (ru, rd, ku, kd) in enumerate(meta["cases"]):
        up, dn = UpSample1d(ru, ku), DownSample1d(rd, kd)
        assert np.array_equal(up.filter.numpy(), g[f"up_filter_c{ci}"]), ci
        assert np.array_equal(dn.lowpass.filter.numpy(), g[f"down_filter_c{ci}"]), ci
        for T in meta["T"]:
            k = f"c{ci}_T{T}"
            sd = {"act.alpha": torch.from_numpy(g[f"alpha_{k}"]), "act.beta": torch.from_numpy(g[f"beta_{k}"]),
                  "upsample.filter": up.filter, "downsample.lowpass.filter": dn.lowpass.filter}
            y = O.activation(torch.from_numpy(g[f"x_{k}"]), sd, "", True, ru, rd)
            assert torch.equal(y, torch.from_numpy(g[f"y_{k}"])), k


def test_vq_fixture_torch_oracle(golden):
    g = golden("vq_decode_latents.npz")
    z = torch.from_numpy(g["z_e"])
    _, idx = O.decode_latents(z.t().reshape(1, 8, -1), torch.from_numpy(g["codebook"]))
    assert torch.equal(idx.reshape(-1), torch.from_numpy(g["indices"]))


def test_vq_fixture_c_oracle(golden):
    g = golden("vq_decode_latents.npz")
    idx = vq_c.argmin(g["z_e"], g["codebook"])
    assert np.array_equal(idx, g["indices"])
    # the planted exact tie resolves to the lower index, like torch's max()
    assert idx[0] == 5


def test_c_oracle_on_model_latents(golden):
    """The C search reproduces the reference's end-to-end codes given the reference's z_e."""
    for fname in MODEL_FILES:
        g = golden(fname)
        meta = g["meta"]
        _, _, _, dsd, _, _ = build_models(meta["model"], **meta["overrides"])
        ze = g["z_e"]  # (B, 8, F)
        idx = vq_c.argmin(ze.transpose(0, 2, 1).reshape(-1, 8), dsd["quantizer.layers.0._codebook.weight"])
        assert np.array_equal(idx, g["codes"][0].reshape(-1)), fname


FSQ_FILES = sorted(f for f in os.listdir(GOLDEN) if f.startswith("fsq_"))


@pytest.mark.parametrize("fname", FSQ_FILES)
def test_fsq_fixture(golden, fname):
    """The FSQ restatement (fsq=True decoders) reproduces the reference's vendored lucidrains FSQ bit for bit
    (tools/make_golden_fsq.py), and the decoder restatement its waveform."""
    from helpers import build_models

    g = golden(fname)
    meta = g["meta"]
    _, dec, _, dsd, _, dk = build_models(meta["model"], **meta["overrides"])
    assert sorted(k for k in dec.state_dict() if k.startswith("quantizer.")) == \
        ["quantizer.project_in.bias", "quantizer.project_in.weight", "quantizer.project_out.bias",
         "quantizer.project_out.weight"]
    sd = torch_sd(dsd)
    with torch.no_grad():
        post, idx = O.fsq_forward(torch.from_numpy(g["z"]), sd, meta["levels"])
        wav = O.decoder_forward(post, sd, dk)
    assert idx.dtype == torch.int32 and torch.equal(idx, torch.from_numpy(g["codes"]))
    assert torch.equal(post, torch.from_numpy(g["post"]))
    assert torch.equal(wav, torch.from_numpy(g["wav"]))
    # token -> latent: indices_to_codes of the reference's own indices and of wrapped / negative integers
    tok = O.fsq_indices_to_codes(torch.from_numpy(g["codes"]), sd, meta["levels"])
    assert torch.equal(tok, torch.from_numpy(g["tok_post"]))
    wrap = O.fsq_indices_to_codes(torch.from_numpy(g["wrap_idx"]), sd, meta["levels"])
    assert torch.equal(wrap, torch.from_numpy(g["wrap_post"]))


@pytest.mark.parametrize("nq", [2, 4])
def test_rvq_multi_quantizer_fixture(golden, nq):
    """ResidualVQ with vq_num_quantizers > 1 (residual_vq.py:21-40): the oracle's residual loop
    reproduces the reference's codes (Nq, B, F), post-VQ embedding, losses and vq2emb bit for bit."""
    g = golden(f"rvq_base_nq{nq}.npz")
    meta = g["meta"]
    _, _, esd, dsd, ek, dk = build_models("base", vq_num_quantizers=nq)
    dsd = torch_sd(dsd)
    with torch.no_grad():
        lat = torch.from_numpy(g["latent"])
        post, codes, losses = O.rvq_forward(lat, dsd, "quantizer.", nq)
        assert codes.shape == (nq, meta["n_clips"], meta["n_samples"] // 200)
        assert torch.equal(codes, torch.from_numpy(g["codes"]))
        assert torch.equal(post, torch.from_numpy(g["post"]))
        assert torch.equal(losses, torch.from_numpy(g["losses"]))
        emb = O.vq2emb(codes.permute(1, 2, 0), dsd, "quantizer.", nq)
        assert torch.equal(emb, torch.from_numpy(g["vq2emb"]))


def test_full_size_fixtures_are_consistent(golden):
    """The full-size reference fixtures (tools/make_golden_full.py) have the shapes the GPU tests and
    bench.py assume; the smallest fp64 top-2 gap is above helpers.GAP_TOL, so a flip anywhere fails."""
    from helpers import GAP_TOL

    g = golden("full_config2_default.npz")
    assert g["codes"].shape == (64, 1200) and g["codes"].dtype == np.int16 and g["gap"].shape == (64, 1200)
    assert g["latent0"].shape == (1024, 1200) and g["latent_fp"].shape == (64, 16)
    assert float(g["gap"].min()) > GAP_TOL
    g3 = golden("full_config3_default.npz")
    assert g3["wav01"].shape == (2, 240000) and g3["wav_fp"].shape == (64, 16)
    l30 = golden("long30_default.npz")
    assert l30["codes"].shape == (3600,) and l30["latent_tail"].shape == (1024, 64)


def test_full_size_fixture_first_clip_against_oracle(golden):
    """Clip 0 of the config-2 fixture re-encoded by the CPU oracle: the same 1200 indices and latent bits
    (the oracle is pinned at full size, not only on the 1 s goldens)."""
    from audiotokenization_amd import synth

    g = golden("full_config2_default.npz")
    _, _, esd, dsd, ek, dk = build_models("default")
    torch.set_num_threads(8)
    x = torch.from_numpy(synth.synth_clips(1, 240000, clip0=0)).unsqueeze(1)
    with torch.no_grad():
        codes, lat = O.encode_indices(x, torch_sd(esd), torch_sd(dsd), ek, dk)
    assert torch.equal(lat[0], torch.from_numpy(g["latent0"]))
    assert np.array_equal(codes[0, 0].numpy().astype(np.int16), g["codes"][0])
