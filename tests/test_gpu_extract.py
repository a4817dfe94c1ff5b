"""Config 4's product loop on the GPU (world 1): extract.extract_sharded with the .npy sink
(extract_indices.py:512-561 layout) equals the per-clip encode, clip for clip."""
import os

import numpy as np
import pytest
import torch

from helpers import build_models

pytestmark = pytest.mark.gpu


def test_extract_sharded_world1_writes_per_clip_npy(dev, tmp_path):
    from audiotokenization_amd.extract import extract_sharded, save_indices, synth_batch

    enc, dec, *_ = build_models("base", device=dev)
    n_clips, T, batch = 7, 12000, 3
    files = {}

    def model(x):
        return dec(enc(x), vq=True)[1]

    def sink(cid, arr):
        files[cid] = save_indices(str(tmp_path), "train-clean-100", f"{100 + cid}_{cid}_000001_000000", arr)

    with torch.no_grad():
        st = extract_sharded(model, n_clips, T, batch, device=dev, sink=sink)
        ref = [dec(enc(synth_batch(1, T, c, dev)), vq=True)[1] for c in range(n_clips)]
        torch.cuda.synchronize()
    assert st.clips == n_clips and st.errors == 0 and st.batches == 3 and sorted(files) == list(range(n_clips))
    for c in range(n_clips):
        path = files[c]
        assert path == os.path.join(str(tmp_path), "train-clean-100", str(100 + c), str(c),
                                    f"{100 + c}_{c}_000001_000000.npy")
        arr = np.load(path)
        assert arr.dtype == np.int16 and arr.shape == (T // 200, 1)
        np.testing.assert_array_equal(arr[:, 0], ref[c][0, 0].cpu().numpy().astype(np.int16))
