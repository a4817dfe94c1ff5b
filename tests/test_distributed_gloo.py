"""Clip-sharded data parallelism on CPU with gloo, world size 2 (the RCCL path's logic):
block partition + per-batch all-gather of the index tensor."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from audiotokenization_amd.extract import all_gather_codes, shard_range

    n_clips, batch, F = 10, 3, 5
    lo, hi = shard_range(n_clips, rank, world)
    per_rank = max(shard_range(n_clips, r, world)[1] - shard_range(n_clips, r, world)[0] for r in range(world))
    got = {}
    for bi in range((per_rank + batch - 1) // batch):
        ids = torch.arange(lo + bi * batch, lo + bi * batch + batch)
        codes = (ids[None, :, None] * 100 + torch.arange(F)[None, None, :]).to(torch.int64)  # fake (1,B,F)
        g = all_gather_codes(codes)
        assert g.shape == (world, 1, batch, F)
        for r in range(world):
            rlo, rhi = shard_range(n_clips, r, world)
            for j in range(batch):
                cid = rlo + bi * batch + j
                if cid < rhi:
                    got[cid] = g[r, 0, j].tolist()
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_all_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        got = results[r]
        assert sorted(got) == list(range(10))
        for cid, row in got.items():
            assert row == [cid * 100 + f for f in range(5)]
