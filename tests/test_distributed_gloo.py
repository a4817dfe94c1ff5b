"""Clip-sharded data parallelism on CPU with gloo, world size 2 (the RCCL path's logic):
block partition + per-batch all-gather of the index tensor."""
import os
import socket

import numpy as np
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


def _run(target, world, *extra):
    # (8 ranks: the spawned interpreters import torch concurrently; the queue wait covers that)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + extra) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return results


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_all_gather(world):
    results = _run(_worker, world)
    for r in range(world):
        got = results[r]
        assert sorted(got) == list(range(10))
        for cid, row in got.items():
            assert row == [cid * 100 + f for f in range(5)]


N_CLIPS, BATCH, NQ, NF = 11, 3, 2, 4


def _fake_source(clip0, n):
    """(n, 1, T) whose sample 0 carries the global clip id (the fake model reads it back)."""
    x = torch.zeros((n, 1, 8))
    x[:, 0, 0] = torch.arange(clip0, clip0 + n, dtype=torch.float32)
    return x


def _fake_codes(ids):
    ids = torch.as_tensor(ids, dtype=torch.int64)
    return ids[None, :, None] * 100 + torch.arange(NQ)[:, None, None] * 10 + torch.arange(NF)[None, None, :]


def _extract_worker(rank, world, port, q, fail_rank, fail_batch, n_clips=N_CLIPS):
    """extract_sharded itself (the product function) with a fake model that raises on one rank's batch."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from audiotokenization_amd.extract import extract_sharded

    calls = {"n": 0}

    def model(x):
        bi = calls["n"]
        calls["n"] += 1
        if rank == fail_rank and bi == fail_batch:
            raise RuntimeError("injected failure")
        return {"indices": _fake_codes(x[:, 0, 0].long())}

    sunk = {}
    st = extract_sharded(model, n_clips, 8, BATCH, rank=rank, world=world, device=torch.device("cpu"),
                         sink=lambda cid, arr: sunk.__setitem__(cid, arr.copy()), source=_fake_source)
    q.put((rank, (st, sunk)))
    dist.barrier()
    dist.destroy_process_group()


# (8, 5, 1, 37): the world config 4 names (8 ranks), 37 clips -> 4 or 5 per rank in batches of 3, so every rank's last
# batch is short (1 or 2 clips) and rank 5's second -- its short last batch -- fails
@pytest.mark.parametrize("world,fail_rank,fail_batch,n_clips", [(2, 1, 0, N_CLIPS), (3, 0, 0, N_CLIPS),
                                                                (3, 2, 1, N_CLIPS), (8, 5, 1, 37), (8, 0, 0, 37)])
def test_extract_sharded_survives_a_failed_batch(world, fail_rank, fail_batch, n_clips):
    """a rank whose batch raises must still join the batch's collectives, so the
    job finishes; the failure is counted (extract_indices.py:565-574) and every other clip arrives."""
    from audiotokenization_amd.extract import shard_range

    results = _run(_extract_worker, world, fail_rank, fail_batch, n_clips)
    flo, fhi = shard_range(n_clips, fail_rank, world)
    lost = list(range(flo + fail_batch * BATCH, min(flo + (fail_batch + 1) * BATCH, fhi)))
    assert lost, "the injected batch must hold real clips"
    if world == 8:  # uneven shards and short last batches, as asked
        sizes = [shard_range(n_clips, r, world)[1] - shard_range(n_clips, r, world)[0] for r in range(world)]
        assert len(set(sizes)) == 2 and all(sz % BATCH for sz in sizes), sizes
    for r in range(world):
        st, sunk = results[r]
        lo, hi = shard_range(n_clips, r, world)
        assert st.errors == (len(lost) if r == fail_rank else 0)
        assert st.error_items == (lost if r == fail_rank else [])
        assert st.clips == hi - lo - st.errors
        assert st.job_errors == len(lost) and st.job_clips == n_clips - len(lost)
        if r == 0:
            assert sorted(sunk) == [c for c in range(n_clips) if c not in lost]
            for cid, arr in sunk.items():
                assert arr.dtype == np.int16 and arr.shape == (NF, NQ)
                np.testing.assert_array_equal(arr, _fake_codes([cid])[:, 0, :].T.numpy())
        else:
            assert sunk == {}


def _all_fail_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from audiotokenization_amd.extract import extract_sharded

    def model(x):
        raise RuntimeError("every batch fails")

    st = extract_sharded(model, 5, 8, 2, rank=rank, world=world, device=torch.device("cpu"), sink=lambda *a: None,
                         source=_fake_source)
    q.put((rank, st))
    dist.barrier()
    dist.destroy_process_group()


def test_extract_sharded_all_ranks_fail():
    results = _run(_all_fail_worker, 2)
    for r, st in results.items():
        assert st.clips == 0 and st.job_errors == 5 and st.job_clips == 0


def test_extract_sharded_single_process_no_dist():
    """world = 1 without an initialised process group: same bookkeeping, no collective."""
    from audiotokenization_amd.extract import extract_sharded

    sunk = {}
    st = extract_sharded(lambda x: _fake_codes(x[:, 0, 0].long()), 7, 8, 3, device=torch.device("cpu"),
                         sink=lambda cid, arr: sunk.__setitem__(cid, arr), source=_fake_source)
    assert st.clips == 7 and st.errors == 0 and st.batches == 3 and sorted(sunk) == list(range(7))


def _shape_worker(rank, world, port, q, odd_rank, odd_batch):
    """A rank whose model returns codes of ANOTHER frame count for one batch (it used to raise
    before the codes gather while the other ranks blocked in it)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from audiotokenization_amd.extract import extract_sharded

    calls = {"n": 0}

    def model(x):
        bi = calls["n"]
        calls["n"] += 1
        c = _fake_codes(x[:, 0, 0].long())
        if rank == odd_rank and bi == odd_batch:
            c = torch.cat([c, c[..., :1]], dim=-1)  # F + 1 frames
        return c

    sunk = {}
    st = extract_sharded(model, N_CLIPS, 8, BATCH, rank=rank, world=world, device=torch.device("cpu"),
                         sink=lambda cid, arr: sunk.__setitem__(cid, arr.copy()), source=_fake_source)
    q.put((rank, (st, sunk)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,odd_rank,odd_batch", [(2, 1, 0), (3, 1, 1), (3, 0, 0)])
def test_extract_sharded_rank_with_other_frame_count(world, odd_rank, odd_batch):
    """Every rank decides the codes gather's shape from the gathered status table (the shape most ranks
    have; ties: the lowest rank's), so the job finishes; the odd rank's batch is counted as failed on
    every rank and every other clip arrives with its own codes."""
    from audiotokenization_amd.extract import shard_range

    results = _run(_shape_worker, world, odd_rank, odd_batch)
    olo, ohi = shard_range(N_CLIPS, odd_rank, world)
    lost = list(range(olo + odd_batch * BATCH, min(olo + (odd_batch + 1) * BATCH, ohi)))
    assert lost
    for r in range(world):
        st, sunk = results[r]
        assert st.errors == (len(lost) if r == odd_rank else 0)
        assert st.job_errors == len(lost) and st.job_clips == N_CLIPS - len(lost)
        if r == 0:
            assert sorted(sunk) == [c for c in range(N_CLIPS) if c not in lost]
            for cid, arr in sunk.items():
                np.testing.assert_array_equal(arr, _fake_codes([cid])[:, 0, :].T.numpy())


def test_agreed_shape_rule():
    from audiotokenization_amd.extract import agreed_shape

    t = torch.tensor([[1, 1, 5, 3], [1, 1, 6, 3], [1, 1, 6, 2], [0, 0, 0, 3]])
    nq, nf, keep = agreed_shape(t)
    assert (nq, nf) == (1, 6) and keep.tolist() == [False, True, True, False]
    nq, nf, keep = agreed_shape(torch.tensor([[1, 2, 7, 1], [1, 2, 8, 1]]))
    assert (nq, nf) == (2, 7) and keep.tolist() == [True, False]
    assert agreed_shape(torch.tensor([[0, 0, 0, 4], [0, 0, 0, 4]])) is None


def test_sink_errors_surface():
    """A sink that raises (e.g. a full disk) fails the extraction on the caller's thread."""
    from audiotokenization_amd.extract import extract_sharded

    def bad_sink(cid, arr):
        raise OSError("disk full")

    with pytest.raises(OSError, match="disk full"):
        extract_sharded(lambda x: _fake_codes(x[:, 0, 0].long()), 7, 8, 3, device=torch.device("cpu"), sink=bad_sink,
                        source=_fake_source)


def test_extract_pipeline_finishes_batch_i_after_queueing_i_plus_1():
    """step(i) queues batch i, then finishes batch i - depth (its status read waits for that batch only, while
    batch i is already queued on the device); flush() finishes the rest.  depth = 0 finishes every batch in
    its own step."""
    from audiotokenization_amd.extract import ShardedExtractor

    log = []

    def model(x):
        log.append(("encode", int(x[0, 0, 0])))
        return _fake_codes(x[:, 0, 0].long())

    def sink(cid, arr):
        log.append(("sink", cid))

    ex = ShardedExtractor(model, 7, 8, 3, device=torch.device("cpu"), sink=sink, source=_fake_source, depth=1)
    assert ex.step(0) is None  # queued only
    g0 = ex.step(1)  # batch 0 finished after batch 1 was queued
    assert g0 is not None and g0.shape == (1, NQ, 3, NF) and g0[0, 0, :, 0].tolist() == [0, 100, 200]
    g1 = ex.step(2)
    assert g1[0, 0, :, 0].tolist() == [300, 400, 500]
    g2 = ex.flush()
    assert g2[0, 0, :, 0].tolist() == [600, 700, 800]  # clips 7, 8 pad the last batch (encoded, never sunk)
    ex.close()
    enc = [c for k, c in log if k == "encode"]
    assert enc == [0, 3, 6]
    assert sorted(c for k, c in log if k == "sink") == list(range(7))
    ex0 = ShardedExtractor(model, 7, 8, 3, device=torch.device("cpu"), source=_fake_source, depth=0)
    assert ex0.step(0)[0, 0, :, 0].tolist() == [0, 100, 200]


def test_extract_deferred_status_word_fails_its_batch():
    """A persistent-kernel status word raised by a forward (deferred into the batch's StatusTicket) fails that
    batch only: counted, not sunk, the other batches arrive (extract_indices.py:565-574)."""
    from audiotokenization_amd import _lib as L
    from audiotokenization_amd.extract import extract_sharded

    calls = {"n": 0}

    def model(x):
        bi = calls["n"]
        calls["n"] += 1
        with L.status_scope():
            L.defer_status(torch.tensor([3 if bi == 1 else 0], dtype=torch.int32), "ResLSTM(test)")
            L.check_status()
        return _fake_codes(x[:, 0, 0].long())

    sunk = {}
    st = extract_sharded(model, 7, 8, 3, device=torch.device("cpu"), sink=lambda cid, arr: sunk.__setitem__(cid, arr),
                         source=_fake_source)
    assert st.errors == 3 and st.error_items == [3, 4, 5] and st.clips == 4
    assert sorted(sunk) == [0, 1, 2, 6]
    with pytest.raises(L.BigCodecLibraryError, match="timed out"):  # outside the deferral the read raises at once
        with L.status_scope():
            L.defer_status(torch.tensor([1], dtype=torch.int32), "ResLSTM(test)")
            L.check_status()


def test_sink_error_stops_the_writer_thread():
    """after a sink error the writer thread is stopped (sentinel + join), not left blocked."""
    import threading

    from audiotokenization_amd.extract import extract_sharded

    def bad_sink(cid, arr):
        raise OSError("disk full")

    with pytest.raises(OSError, match="disk full"):
        extract_sharded(lambda x: _fake_codes(x[:, 0, 0].long()), 7, 8, 3, device=torch.device("cpu"), sink=bad_sink,
                        source=_fake_source)
    assert not [t for t in threading.enumerate() if t.name == "bigcodec-sink" and t.is_alive()]
