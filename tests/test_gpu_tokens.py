"""Token -> audio service path (audiotokenization_amd/tokens.py, bc_vq2emb_ct)
against the CPU oracle on the same codes.

Tolerances (fp32): embedding max|d| / max|ref| <= 1e-6 (the K = 8 out_proj in a different fp32 order than
MKL's sgemm; our own vq2emb kernel is the bit-exact reference for the layout change); waveform MSE <= 1e-12
and max|d| <= 1e-5, the decoder bound of test_gpu_model.py.
"""
import os

import numpy as np
import pytest
import torch

from audiotokenization_amd import extract, tokens
from helpers import assert_close_rel, build_models, torch_sd
from oracle import bigcodec_oracle as O

pytestmark = pytest.mark.gpu


def _codes(dec, B, F, nq, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, dec.quantizer.layers[0].codebook_size, (B, F, nq), generator=g)


@pytest.mark.parametrize("model,nq,F", [("debug", 1, 37), ("debug", 2, 50), ("base", 1, 24), ("debug", 3, 1)])
def test_tokens_to_audio_matches_oracle(dev, model, nq, F):
    _, dec, _, dsd, _, dk = build_models(model, device=dev, vq_num_quantizers=nq)
    codes = _codes(dec, 2, F, nq, seed=7 * nq + F)
    sd = torch_sd(dsd)
    with torch.no_grad():
        ref_emb = O.vq2emb(codes, sd, "quantizer.", nq)  # (B, F, D)
        ref_wav = O.decoder_forward(ref_emb.transpose(1, 2).contiguous(), sd, dk)
        emb = dec.quantizer.vq2emb_ct(codes.to(dev))
        own = dec.vq2emb(codes.to(dev).contiguous())
        wav = dec.tokens_to_audio(codes.to(dev))
        torch.cuda.synchronize()
    assert emb.shape == (2, ref_emb.shape[2], F)
    assert torch.equal(emb.cpu(), own.cpu().transpose(1, 2)), "bc_vq2emb_ct != bc_vq2emb (+ transpose)"
    assert_close_rel(emb.cpu(), ref_emb.transpose(1, 2), 1e-6, "vq2emb_ct")
    w, r = wav.cpu().double(), ref_wav.double()
    assert w.shape == r.shape == (2, 1, F * dec.hop_length)
    mse, mx = float(((w - r) ** 2).mean()), float((w - r).abs().max())
    print(f"tokens->audio {model} nq={nq} F={F}: mse {mse:.2e} max {mx:.2e}")
    assert mse <= 1e-12 and mx <= 1e-5


def test_out_of_range_index_gives_nan_not_a_fault(dev):
    _, dec, _, _, _, _ = build_models("debug", device=dev)
    codes = _codes(dec, 1, 8, 1, seed=3)
    codes[0, 5, 0] = dec.quantizer.layers[0].codebook_size  # one past the end
    codes[0, 2, 0] = -1
    emb = dec.quantizer.vq2emb_ct(codes.to(dev)).cpu()
    bad = torch.isnan(emb).all(dim=1)[0]
    assert bad.tolist() == [i in (2, 5) for i in range(8)]


def test_decode_index_files_round_trip(dev, tmp_path):
    """extract.save_indices files (int16 (F, 1)) of ragged lengths decode, batched by length, to exactly
    what decoding each clip alone gives."""
    _, dec, _, _, _, _ = build_models("debug", device=dev)
    paths = []
    for i, F in enumerate([20, 33, 20, 33, 7]):
        c = _codes(dec, 1, F, 1, seed=100 + i)
        paths.append(extract.save_indices(str(tmp_path), "test-clean", f"{i}-1-{i:04d}", c[0].numpy().astype(np.int16)))
    wavs = tokens.decode_index_files(dec, paths, dev, batch=2)
    for p, w in zip(paths, wavs):
        arr = tokens.load_indices(p)
        alone = dec.tokens_to_audio(torch.from_numpy(arr.astype(np.int64))[None].to(dev)).cpu().numpy()[0, 0]
        assert w.shape == (arr.shape[0] * dec.hop_length,)
        assert np.array_equal(w, alone), os.path.basename(p)
