"""Host logic: synthetic weight / clip spec, index post-processing and file layout (extract_indices.py
:512-561), clip sharding."""
import os

import numpy as np
import pytest
import torch

from audiotokenization_amd import synth
from audiotokenization_amd.extract import (batch_indices_to_numpy, batches, indices_to_numpy, output_path,
                                           parse_fileid, save_indices, shard_range)


def test_synth_clips_formula():
    x = synth.synth_clips(3, 1000, clip0=5)
    assert x.dtype == np.float32 and x.shape == (3, 1000)
    assert x.min() >= -0.5 and x.max() < 0.5
    i, n = 6, 123
    h = synth.splitmix64(np.uint64(0xB16C0DEC) ^ (np.uint64(i) << np.uint64(32)) ^ np.uint64(n))
    assert x[1, n] == np.float32(int(h) >> 40) / np.float32(1 << 24) - np.float32(0.5)
    assert np.array_equal(synth.synth_clips(3, 1000, clip0=5), x)
    assert abs(float(x.mean())) < 0.02


def test_splitmix64_reference_values():
    # splitmix64 finaliser of 0 (x + golden gamma, then mix) — standard first output of seed 0
    assert int(synth.splitmix64(np.uint64(0))) == 0xE220A8397B1DCDAF


def test_synth_state_dict_deterministic_and_complete():
    from audiotokenization_amd import preset
    from audiotokenization_amd.lightning_shim import CodecLightningModule

    lm = CodecLightningModule(preset("debug", antialias=True))
    sd = lm.state_dict()
    a = synth.synth_state_dict(sd)
    b = synth.synth_state_dict(sd)
    assert set(a) == set(sd)
    for k in a:
        assert a[k].shape == tuple(sd[k].shape) and np.array_equal(a[k], b[k]), k
    g = a["encoder.block.0.weight_g"].reshape(-1)
    v = a["encoder.block.0.weight_v"].reshape(g.shape[0], -1)
    ratio = g / np.linalg.norm(v.astype(np.float64), axis=1)
    assert ratio.min() >= 0.74 and ratio.max() <= 1.26
    assert np.array_equal(a["encoder.block.1.block.0.block.0.upsample.filter"],
                          sd["encoder.block.1.block.0.block.0.upsample.filter"].numpy())


def test_indices_to_numpy_matches_reference_postprocessing():
    codes = torch.tensor([[[7, 8, 9, 8191]]], dtype=torch.int64)  # (Nq=1, B=1, F=4)
    arr = indices_to_numpy(codes)
    assert arr.dtype == np.int16 and arr.shape == (4, 1) and arr[:, 0].tolist() == [7, 8, 9, 8191]
    # (1, F): squeeze(1) is a no-op there, so the reference permutes it to (F, 1) as well
    arr1 = indices_to_numpy(torch.tensor([[1, 2, 3]]))
    assert arr1.shape == (3, 1)
    multi = torch.arange(24).reshape(2, 3, 4)  # (Nq=2, B=3, F=4)
    bb = batch_indices_to_numpy(multi)
    assert bb.shape == (3, 4, 2)
    for b in range(3):
        assert np.array_equal(bb[b], indices_to_numpy(multi[:, b:b + 1]))
    with pytest.raises(ValueError):
        indices_to_numpy(torch.zeros(2, 1, 2, 2))


def test_output_layout(tmp_path):
    assert parse_fileid("1034_121119_000001_000001") == ("1034", "121119")
    assert parse_fileid("84-121123-0000") == ("84", "121123")
    assert parse_fileid("weird") == ("unknown", "unknown")
    p = output_path(str(tmp_path), "dev-clean", "84-121123-0000")
    assert p == os.path.join(str(tmp_path), "dev-clean", "84", "121123", "84-121123-0000.npy")
    arr = np.arange(10, dtype=np.int16).reshape(10, 1)
    path = save_indices(str(tmp_path), "dev-clean", "84-121123-0000", arr)
    assert np.array_equal(np.load(path), arr)


@pytest.mark.parametrize("n,w", [(100000, 8), (10, 3), (7, 8), (64, 1)])
def test_shard_range_partitions(n, w):
    seen = []
    for r in range(w):
        lo, hi = shard_range(n, r, w)
        assert 0 <= lo <= hi <= n
        seen.extend(range(lo, hi))
        assert hi - lo in (n // w, n // w + 1)
    assert seen == list(range(n))
    assert batches(0, 10, 4) == [(0, 4), (4, 8), (8, 10)]


def test_token_files_host_side(tmp_path):
    """tokens.py host logic (no GPU): extract.save_indices files load back, stack ragged with padding and
    lengths, int16 codes >= 32768 wrap back, out-of-range codes and mixed quantizer counts raise."""
    import pytest

    from audiotokenization_amd import extract, tokens

    a = np.array([[0], [5], [8191]], dtype=np.int16)
    b = np.array([[3], [4]], dtype=np.int16)
    pa = extract.save_indices(str(tmp_path), "dev-clean", "1-2-0003", a)
    pb = extract.save_indices(str(tmp_path), "dev-clean", "1-2-0004", b)
    la, lb = tokens.load_indices(pa), tokens.load_indices(pb)
    assert la.dtype == np.int16 and np.array_equal(la, a)
    codes, lengths = tokens.codes_to_device([la, lb], "cpu", 8192)
    assert lengths == [3, 2] and codes.dtype == torch.int64 and codes.shape == (2, 3, 1)
    assert codes[:, :, 0].tolist() == [[0, 5, 8191], [3, 4, 0]]
    big = np.array([[40000 - 65536]], dtype=np.int16)  # a 65536-entry codebook's index 40000, as int16
    assert tokens.codes_to_device([big], "cpu", 65536)[0].item() == 40000
    with pytest.raises(ValueError):
        tokens.codes_to_device([np.array([[8192]], dtype=np.int16)], "cpu", 8192)
    with pytest.raises(ValueError):
        tokens.codes_to_device([a, np.zeros((2, 2), dtype=np.int16)], "cpu", 8192)
