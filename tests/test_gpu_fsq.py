"""FSQ quantizer (decoder fsq=True) on the MI355X against the reference's own
outputs (tests/golden/fsq_*.npz from tools/make_golden_fsq.py; the oracle reproduces them bit for bit,
test_oracle_pinned.py::test_fsq_fixture).

Tolerances: indices equal except frames whose fp64 distance from a coordinate to its rounding boundary
(`margin`) is below 1e-4 (project_in's 512/1024-term sum runs in a different fp32 order than MKL's);
quantized output max|d| / max|ref| <= 1e-6 on the frames with equal indices (a function of the codes
only); decoded waveform MSE <= 1e-12, max|d| <= 1e-5 (test_gpu_model.py's decoder bound).
"""
import os

import numpy as np
import pytest
import torch

from helpers import assert_close_rel, build_models

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FSQ_FILES = sorted(f for f in os.listdir(GOLDEN) if f.startswith("fsq_"))


@pytest.mark.parametrize("fname", FSQ_FILES)
def test_fsq_decoder_against_reference(dev, golden, fname):
    g = golden(fname)
    meta = g["meta"]
    _, dec, *_ = build_models(meta["model"], device=dev, **meta["overrides"])
    with torch.no_grad():
        post, q, loss = dec(torch.from_numpy(g["z"]).to(dev), vq=True)
        wav = dec(torch.from_numpy(g["post"]).to(dev), vq=False)
        torch.cuda.synchronize()
    assert q.dtype == torch.int32 and tuple(q.shape) == g["codes"].shape
    assert float(loss.abs().sum()) == 0.0 and tuple(loss.shape) == (g["z"].shape[0],)
    qc = q.cpu().numpy()
    bad = np.nonzero(qc != g["codes"])
    worst = float(g["margin"][bad].max()) if bad[0].size else 0.0
    print(f"{fname}: {bad[0].size} index mismatches of {qc.size} (worst margin {worst:.2e}), "
          f"{len(np.unique(qc))} distinct codes")
    assert worst <= 1e-4
    same = torch.from_numpy(qc == g["codes"])[:, None, :].expand(-1, g["post"].shape[1], -1)
    assert_close_rel(post.cpu()[same], torch.from_numpy(g["post"])[same], 1e-6, "fsq post")
    w, r = wav.cpu().double(), torch.from_numpy(g["wav"]).double()
    mse, mx = float(((w - r) ** 2).mean()), float((w - r).abs().max())
    assert mse <= 1e-12 and mx <= 1e-5, (mse, mx)


def test_fsq_identity_projection_and_all_codes(dev):
    """dim == len(levels) (no projections): every one of the prod(levels) grid points maps to its own
    index, in codes_to_indices' mixed-radix order, exactly as the restatement computes it."""
    from audiotokenization_amd.modules import FSQ
    from oracle import bigcodec_oracle as O

    levels = [8, 5, 5, 5]
    m = FSQ(levels, dim=4, channel_first=True).eval()
    lv = torch.tensor(levels, dtype=torch.float64)
    grid = torch.stack(torch.meshgrid(*[torch.arange(v, dtype=torch.float64) for v in levels], indexing="ij"), -1)
    grid = grid.reshape(-1, 4)  # level index per coordinate
    half_l = (lv - 1) * 1.001 / 2
    offset = torch.where(lv % 2 == 0, 0.5, 0.0).double()
    shift = torch.atanh(offset / half_l)
    target = grid - torch.div(lv, 2, rounding_mode="floor")  # the bounded value that rounds to this point
    z = (torch.atanh(((target + offset) / half_l).clamp(-0.999999, 0.999999)) - shift).float()
    z = z.t().contiguous()[None]  # (1, 4, 1000)
    with torch.no_grad():
        post, q = m(z.to(dev))
        ref_post, ref_q = O.fsq_forward(z, {}, levels)
    assert torch.equal(q.cpu(), ref_q)
    assert len(torch.unique(q)) == int(np.prod(levels))
    assert torch.equal(post.cpu(), ref_post)


@pytest.mark.parametrize("fname", FSQ_FILES)
def test_fsq_tokens_to_audio_against_reference(dev, golden, fname, tmp_path):
    """The fsq=True decoder's token -> audio path (FSQ.indices_to_codes, finite_scalar_quantization.py:176-192,
    on bc_fsq_codes; the reference decoder's vq2emb has no FSQ branch and raises AttributeError, as ours does):
      * indices_to_codes of the reference's indices (int32 as forward returns them, and int64 as the token files
        give them) equals this path's own forward post bit for bit and the reference's within 1e-6 of max|ref|
        (project_out: 4-term fma chain vs MKL);
      * out-of-range and negative integers wrap exactly as torch's floor // and % wrap them (reference fixture);
      * tokens -> .npy files -> decode_index_files -> waveform within the decoder bound of the reference's
        waveform (MSE <= 1e-12, max|d| <= 1e-5)."""
    from audiotokenization_amd.extract import save_indices
    from audiotokenization_amd.tokens import decode_index_files

    g = golden(fname)
    meta = g["meta"]
    _, dec, *_ = build_models(meta["model"], device=dev, **meta["overrides"])
    codes = torch.from_numpy(g["codes"])  # (B, F) int32, the reference's indices
    with torch.no_grad():
        post, q, _ = dec(torch.from_numpy(g["z"]).to(dev), vq=True)
        t32 = dec.quantizer.indices_to_codes(codes.to(dev))
        t64 = dec.quantizer.indices_to_codes(codes.long().to(dev))
        wrap = dec.quantizer.indices_to_codes(torch.from_numpy(g["wrap_idx"]).to(dev))
        wrap32 = dec.quantizer.indices_to_codes(torch.from_numpy(g["wrap_idx"]).int().to(dev))
        torch.cuda.synchronize()
    with pytest.raises(AttributeError):
        dec.vq2emb(codes[:, :, None].long().to(dev))
    assert t32.shape == g["tok_post"].shape and torch.equal(t32, t64) and torch.equal(wrap, wrap32)
    same = (q.cpu() == codes).all()
    if bool(same):
        assert torch.equal(t32, post), "indices_to_codes(forward's indices) != forward's post"
    assert_close_rel(t32.cpu(), torch.from_numpy(g["tok_post"]), 1e-6, "fsq indices_to_codes")
    assert_close_rel(wrap.cpu(), torch.from_numpy(g["wrap_post"]), 1e-6, "fsq indices_to_codes (wrapped)")
    paths = [save_indices(str(tmp_path), "fsq", f"1_1_000001_{i:06d}", g["codes"][i][:, None].astype(np.int16))
             for i in range(codes.shape[0])]
    wavs = decode_index_files(dec, paths, dev)
    for i, w in enumerate(wavs):
        r = g["wav"][i, 0].astype(np.float64)
        d = w.astype(np.float64) - r
        mse, mx = float((d ** 2).mean()), float(np.abs(d).max())
        print(f"{fname} clip {i}: tokens -> audio mse {mse:.2e} max {mx:.2e}")
        assert w.shape == r.shape and mse <= 1e-12 and mx <= 1e-5, (mse, mx)
