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


def test_rccl_codes_all_gather_world1(dev):
    """The codes all-gather's collective (extract._all_gather_wire: the int16 byte view, dist.all_gather_into_tensor,
    the reassembly) executed over RCCL on the GPU.  One GPU per box: a world-1 "nccl" group (all_gather_codes itself
    returns early at world 1, so without this the RCCL call never ran on hardware); worlds 2-8 run the same function
    over gloo in tests/test_distributed_gloo.py."""
    import socket

    import torch.distributed as dist

    from audiotokenization_amd.extract import _all_gather_wire

    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device(dev))
    try:
        assert dist.get_backend() == "nccl"
        g = torch.Generator().manual_seed(5)
        for dtype in (torch.int16, torch.int64):
            codes = torch.randint(-32768, 32767, (2, 7, 61), generator=g).to(dtype).to(dev)
            out = _all_gather_wire(codes, 1)
            torch.cuda.synchronize()
            assert out.dtype == dtype and out.shape == (1, 2, 7, 61)
            assert torch.equal(out[0].cpu(), codes.cpu())
    finally:
        dist.destroy_process_group()
