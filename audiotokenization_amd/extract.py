"""extract_indices-equivalent driver (extract_indices.py:281-589) on the HIP path.

  * index post-processing and on-disk format (extract_indices.py:512-561): codes (Nq, 1, F) ->
    squeeze(1) -> permute to (F, Nq) -> int16 -> np.save(<out>/<subset>/<spk>/<chapter>/<fileid>.npy)
  * clip-sharded data-parallel extraction: global clip ids are block-partitioned
    over ranks, each rank encodes its own batches, and the batch's index tensor is all-gathered as
    int16 over the process group (RCCL over xGMI on MI355X, gloo on CPU test runs); the per-batch status
    table travels over a host-side gloo group, so no host waits for an encode while its device idles.
  * per-item error accounting (extract_indices.py:565-574): failures are counted, not fatal.
"""
from __future__ import annotations

import collections
import os
import weakref
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Tuple

import numpy as np
import torch

from . import _lib as L
from . import ops


def indices_to_numpy(indices: torch.Tensor) -> np.ndarray:
    """extract_indices.py:520-532 for one clip: (Nq, 1, F) -> (F, Nq) int16 (or (F,) from (1, F))."""
    indices = indices.squeeze(1)
    if indices.ndim == 2:
        indices = indices.permute(1, 0)
    elif indices.ndim != 1:
        raise ValueError(f"Unexpected indices dimension: {indices.ndim}")
    return indices.cpu().numpy().astype(np.int16)


def batch_indices_to_numpy(codes: torch.Tensor) -> np.ndarray:
    """(Nq, B, F) -> (B, F, Nq) int16; row b equals indices_to_numpy(codes[:, b:b+1])."""
    if codes.ndim != 3:
        raise ValueError("codes must be (Nq, B, F)")
    return codes.permute(1, 2, 0).cpu().numpy().astype(np.int16)


def parse_fileid(fileid: str) -> Tuple[str, str]:
    """extract_indices.py:536-548: speaker / chapter from a LibriTTS / LibriSpeech file id."""
    if "_" in fileid:
        parts = fileid.split("_")
        return parts[0], parts[1]
    if "-" in fileid:
        parts = fileid.split("-")
        return parts[0], parts[1]
    return "unknown", "unknown"


def output_path(output_dir: str, subset: str, fileid: str) -> str:
    """extract_indices.py:551-558."""
    spk, ch = parse_fileid(fileid)
    return os.path.join(output_dir, subset, spk, ch, f"{fileid}.npy")


def save_indices(output_dir: str, subset: str, fileid: str, indices_np: np.ndarray) -> str:
    path = output_path(output_dir, subset, fileid)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    np.save(path, indices_np)
    return path


class BigCodecModel(torch.nn.Module):
    """extract_indices.py:281-371 / inference_full.py:535-561 wrapper around a CodecLightningModule."""

    def __init__(self, lm, reconstruct: bool = False):
        super().__init__()
        self.lm = lm
        self.reconstruct = reconstruct
        self.codebook_size = lm.cfg.model.codec_decoder.codebook_size

    @torch.no_grad()
    def forward(self, x):
        vq_emb = self.lm.model["CodecEnc"](x)
        vq_post_emb, vq_code, _ = self.lm.model["generator"](vq_emb, vq=True)
        if not self.reconstruct:
            return {"indices": vq_code}
        recon = self.lm.model["generator"](vq_post_emb, vq=False)
        return {"x_rec": recon, "indices": vq_code, "loss": {}}


def pad_like_inference_full(x: torch.Tensor, hop: int = 200) -> torch.Tensor:
    """inference_full.py:712: F.pad(x, (0, hop - T % hop)) — always pads (a full hop when T is
    already a multiple).  Allocation + copy only."""
    B, C, T = x.shape
    pad = hop - (T % hop)
    out = torch.zeros((B, C, T + pad), device=x.device, dtype=x.dtype)
    out[..., :T] = x
    return out


# ------------------------------------------------------------------------------------------------
# clip-sharded data-parallel extraction
# ------------------------------------------------------------------------------------------------
def shard_range(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Block partition of [0, n_items): rank r gets [r*n/W, (r+1)*n/W)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    lo = (n_items * rank) // world
    hi = (n_items * (rank + 1)) // world
    return lo, hi


def batches(lo: int, hi: int, batch: int) -> List[Tuple[int, int]]:
    return [(s, min(s + batch, hi)) for s in range(lo, hi, batch)]


def synth_batch(n_clips: int, n_samples: int, clip0: int, device) -> torch.Tensor:
    """White-noise clips (B, 1, T) generated in HBM by bc_synth_clips (same values as synth.synth_clips)."""
    x = torch.empty((n_clips, 1, n_samples), device=device, dtype=torch.float32)
    if not x.is_cuda:
        raise L.BigCodecLibraryError("synth_batch generates clips on a HIP device")
    ops.load().synth_clips_(x, clip0)
    return x


def all_gather_codes(codes: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather one batch's (Nq, B, F) int64 / int16 codes over the process group -> (W, Nq, B, F).
    Ranks must pass equal shapes (pad the last batch)."""
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return codes.unsqueeze(0)
    return _all_gather_wire(codes, dist.get_world_size(group), group)


def _all_gather_wire(codes: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """The collective of all_gather_codes (also run at world 1 by tests/test_gpu_extract.py, so the RCCL call, the int16
    byte view and the reassembly execute on a GPU): (Nq, B, F) per rank -> (W, Nq, B, F)."""
    import torch.distributed as dist

    codes = codes.contiguous()
    # int16 (the on-disk type) travels as its bytes: RCCL and gloo have no 16-bit integer type
    wire = codes.view(torch.int8) if codes.dtype == torch.int16 else codes
    out = torch.empty((world * wire.shape[0],) + tuple(wire.shape[1:]), dtype=wire.dtype, device=wire.device)
    dist.all_gather_into_tensor(out, wire, group=group)
    return out.view(codes.dtype).view((world,) + tuple(codes.shape))


def all_gather_status(status: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather a small int64 status vector per rank -> (W, n)."""
    import torch.distributed as dist

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return status.unsqueeze(0)
    world = dist.get_world_size(group)
    out = torch.empty((world * status.numel(),), dtype=status.dtype, device=status.device)
    dist.all_gather_into_tensor(out, status.contiguous(), group=group)
    return out.view(world, status.numel())


@dataclass
class ExtractStats:
    clips: int = 0          # this rank's clips encoded
    errors: int = 0         # this rank's clips lost to a failed batch (extract_indices.py:565-574)
    frames: int = 0
    batches: int = 0
    error_items: List[int] = field(default_factory=list)
    job_errors: int = 0     # clips lost on ANY rank (every rank sees the per-batch status gather)
    job_clips: int = 0      # clips encoded on all ranks


def _codes_of(out) -> torch.Tensor:
    return out["indices"] if isinstance(out, dict) else out


def agreed_shape(stat: torch.Tensor):
    """The (Nq, F) the batch's codes all-gather uses, decided from the gathered status table
    stat (W, 4) = (ok, Nq, F, real clips) that EVERY rank holds, so every rank decides the same: the shape
    of the most ok rows (ties: the lowest rank's).  Returns (nq, nf, ok mask of the rows that have it) or
    None when no rank succeeded; an ok row with another shape is treated as a failed batch."""
    ok = stat[:, 0].bool()
    if not bool(ok.any()):
        return None
    shapes = [(int(stat[r, 1]), int(stat[r, 2])) for r in range(stat.shape[0]) if bool(ok[r])]
    best = max(shapes, key=lambda sh: (shapes.count(sh), -shapes.index(sh)))
    keep = ok & (stat[:, 1] == best[0]) & (stat[:, 2] == best[1])
    return best[0], best[1], keep


class _SinkWriter:
    """Rank 0's host side of the extraction, off the critical path: the gathered codes are copied into a
    pinned buffer on a side stream (ordered after the gather by an event), and a writer thread waits for
    that copy, then hands every clip's (F, Nq) int16 array to the sink.  At most `depth` batches are queued;
    errors in the sink are re-raised by flush()."""

    def __init__(self, sink, depth: int = 4):
        import queue
        import threading

        self.sink = sink
        self.q = queue.Queue(maxsize=depth)
        self.err = None
        self.side = None
        self.t = threading.Thread(target=self._loop, name="bigcodec-sink", daemon=True)
        self.t.start()

    def submit(self, gathered: torch.Tensor, rows):
        """gathered (W, Nq, B, F) int16; rows = [(r, [(clip id, column j), ...]), ...] to sink."""
        if self.err is not None:
            raise self.err
        if gathered.is_cuda:
            if self.side is None:
                self.side = torch.cuda.Stream(device=gathered.device)
            host = torch.empty(gathered.shape, dtype=gathered.dtype, pin_memory=True)
            ev = torch.cuda.Event()
            self.side.wait_stream(torch.cuda.current_stream(gathered.device))
            with torch.cuda.stream(self.side):
                host.copy_(gathered, non_blocking=True)
                gathered.record_stream(self.side)
                ev.record(self.side)
        else:
            host, ev = gathered.clone(), None
        self.q.put((host, ev, rows))
        return host

    def _loop(self):
        while True:
            item = self.q.get()
            if item is None:
                self.q.task_done()
                return
            host, ev, rows = item
            try:
                if self.err is None:
                    if ev is not None:
                        ev.synchronize()
                    arr = host.permute(0, 3, 2, 1).numpy()  # (W, F, B, Nq) view: arr[r, :, j] is clip j's (F, Nq)
                    for r, clips in rows:
                        for cid, j in clips:
                            self.sink(cid, np.ascontiguousarray(arr[r, :, j]))
            except BaseException as e:  # surfaced by submit / flush on the caller's thread
                self.err = e
            finally:
                self.q.task_done()

    def flush(self):
        self.q.join()
        if self.err is not None:
            err, self.err = self.err, None
            raise err

    def close(self):
        self.q.put(None)
        self.t.join()


# WORLD group -> {ranks: the gloo control group of ShardedExtractor} (one per process and world; weak keys, so a
# destroyed world's groups are dropped with it)
_CONTROL_GROUPS = weakref.WeakKeyDictionary()


class ShardedExtractor:
    """Clip-sharded extraction of clips [0, n_clips) over `world` ranks.

    Rank r owns the block shard_range(n_clips, r, world) and walks it in batches of `batch`; every
    rank runs the same number of batches (the last ones padded with clip ids that are discarded), so
    the per-batch collectives line up.  A batch whose source or model raises is counted, not fatal
    (extract_indices.py:565-574) — and the failing rank STILL joins both of the batch's collectives:
    first an all-gather of (ok, Nq, F, real clips) per rank, then, if any rank succeeded, the all-gather of
    the (Nq, B, F) codes as int16 (the on-disk type, extract_indices.py:532), in which a failed rank
    contributes zeros of the agreed shape.  The agreed shape comes from the status table every rank holds
    (agreed_shape), so a rank whose codes have another shape is counted as failed on every rank alike
    and no rank can be left waiting in a collective another rank skipped.

    Nothing on the host waits for a batch's encode while the device is idle: step(i) queues batch i's
    encode with its status words deferred (_lib.deferred_status), and only then finishes batch i - `depth`
    (reads its status words — the device is busy with batch i meanwhile —, exchanges the status table over a
    host-side gloo group, queues the codes all-gather over the device group, RCCL on MI355X, and hands the
    codes to the sink).  flush() finishes every queued batch.

    `source(clip0, n) -> (n, 1, T)` supplies a batch (default: bc_synth_clips on `device`);
    `model(x)` returns the codes (Nq, B, F) or a dict with "indices" (BigCodecModel);
    `sink(global_clip_id, codes (F, Nq) int16)` receives every successfully encoded clip of the job
    on rank 0 (e.g. an .npy writer, save_indices), on a writer thread that runs behind the device (the
    D2H copy and the sink overlap the next batches); run() / flush() wait for it."""

    def __init__(self, model, n_clips: int, n_samples: int, batch: int, rank: int = 0, world: int = 1,
                 device=None, gather: bool = True, sink=None, group=None, source=None, sink_depth: int = 4,
                 depth: int = 1):
        if batch <= 0 or n_clips < 0 or depth < 0:
            raise ValueError("batch must be > 0, n_clips >= 0 and depth >= 0")
        self.model, self.n_clips, self.n_samples, self.batch = model, n_clips, n_samples, batch
        self.rank, self.world, self.gather, self.sink, self.group = rank, world, gather, sink, group
        self.depth = depth
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.source = source or (lambda clip0, n: synth_batch(n, n_samples, clip0, self.device))
        self.lo, self.hi = shard_range(n_clips, rank, world)
        per_rank = max(shard_range(n_clips, r, world)[1] - shard_range(n_clips, r, world)[0] for r in range(world))
        self.n_batches = (per_rank + batch - 1) // batch
        self.stats = ExtractStats()
        self.writer = _SinkWriter(sink, sink_depth) if (rank == 0 and sink is not None) else None
        self.last = None  # rank 0: the last batch's gathered (W, Nq, B, F) int16 host tensor (filled behind the device)
        self.queued = collections.deque()  # batches encoded (queued on the device) but not finished yet
        self.ctl = self._control_group() if (gather and world > 1) else None

    def _control_group(self):
        """The host-side group of the status exchange: the device group itself when it is gloo, else a gloo
        group over the same ranks, created ONCE per process and set of ranks and shared by every extractor (ADVICE
        r04: one new group per extractor was never destroyed, and every rank had to build extractors in the same
        order).  new_group is collective, so the first extractor over a set of ranks is built on every rank."""
        import torch.distributed as dist

        if not dist.is_available() or not dist.is_initialized():
            return None
        if dist.get_backend(self.group) == "gloo":
            return self.group
        ranks = tuple(dist.get_process_group_ranks(self.group)) if self.group is not None else None
        # keyed on the WORLD group object itself (weakly: a destroyed world's entries go with it), not on id(): after
        # destroy_process_group() and a re-init the new WORLD may reuse the freed object's address
        world = dist.group.WORLD
        per_world = _CONTROL_GROUPS.get(world)
        if per_world is None:
            per_world = _CONTROL_GROUPS[world] = {}
        grp = per_world.get(ranks)
        if grp is None:
            grp = per_world[ranks] = dist.new_group(ranks=list(ranks) if ranks else None, backend="gloo")
        return grp

    def step(self, bi: int):
        """Queue batch `bi` of every rank on the device, then finish the batches beyond the pipeline depth.
        Returns the gathered (W, Nq, B, F) int16 device codes of the last batch finished here, or None (no
        batch finished, or it failed on every rank)."""
        s = self.lo + bi * self.batch
        real = max(0, min(s + self.batch, self.hi) - s)
        codes = ticket = None
        try:
            with L.deferred_status() as ticket:
                codes = _codes_of(self.model(self.source(s, self.batch)))
            if codes.ndim != 3 or codes.shape[1] != self.batch:
                raise ValueError(f"model returned codes of shape {tuple(codes.shape)}, expected (Nq, {self.batch}, F)")
        except Exception:  # per-batch accounting, mirrors extract_indices.py:565-574
            codes = None
        self.queued.append((bi, s, real, codes, ticket))
        out = None
        while len(self.queued) > self.depth:
            out = self._finish(*self.queued.popleft())
        return out

    def _finish(self, bi, s, real, codes, ticket):
        st = self.stats
        if codes is not None:
            try:
                ticket.check()  # the batch's persistent-LSTM status words (waits for this batch only)
            except Exception:
                codes = None
        st.batches += 1
        gather = self.gather and self.world > 1
        status = torch.tensor([1 if codes is not None else 0, codes.shape[0] if codes is not None else 0,
                               codes.shape[2] if codes is not None else 0, real], dtype=torch.int64)
        stat = all_gather_status(status, self.ctl) if gather else status.unsqueeze(0)
        agreed = agreed_shape(stat)
        keep = agreed[2] if agreed is not None else torch.zeros(stat.shape[0], dtype=torch.bool)
        me = self.rank if gather else 0
        if bool(keep[me]):
            st.clips += real
            st.frames += real * codes.shape[-1]
        else:  # failed here, or a shape the other ranks do not share: the batch's clips are lost
            codes = None
            st.errors += real
            st.error_items.extend(range(s, s + real))
        st.job_errors += int(stat[~keep, 3].sum())
        st.job_clips += int(stat[keep, 3].sum())
        if agreed is None:
            return None
        nq, nf = agreed[0], agreed[1]
        codes16 = (torch.zeros((nq, self.batch, nf), dtype=torch.int16, device=self.device) if codes is None
                   else codes.to(torch.int16))  # extract_indices.py:532's astype(np.int16), on the device
        gathered = all_gather_codes(codes16, self.group) if gather else codes16.unsqueeze(0)
        if self.writer is not None:
            rows = []
            for r in range(gathered.shape[0]):
                if not bool(keep[r if gather else 0]):
                    continue
                rlo, rhi = shard_range(self.n_clips, r, self.world) if gather else (self.lo, self.hi)
                rs = rlo + bi * self.batch
                rows.append((r, [(rs + j, j) for j in range(self.batch) if rs + j < rhi]))
            self.last = self.writer.submit(gathered, rows)
        return gathered

    def flush(self):
        """Finish every queued batch, then wait until the sink has received them (re-raises a sink error).
        Returns the gathered codes of the last batch finished, or None."""
        out = None
        while self.queued:
            out = self._finish(*self.queued.popleft())
        if self.writer is not None:
            self.writer.flush()
        return out

    def close(self):
        """Stop the writer thread (after it has drained; a sink error is re-raised once it has stopped).
        Batches still queued are not finished: flush() first on the success path."""
        w, self.writer = self.writer, None
        if w is not None:
            try:
                w.flush()
            finally:
                w.close()

    def run(self) -> ExtractStats:
        ok = False
        try:
            for bi in range(self.n_batches):
                self.step(bi)
            self.flush()
            ok = True
        finally:
            if ok:
                self.close()
            else:  # the original exception propagates; a sink error behind it must not replace it
                try:
                    self.close()
                except Exception:
                    pass
        return self.stats


def extract_sharded(model, n_clips: int, n_samples: int, batch: int, rank: int = 0, world: int = 1, device=None,
                    gather: bool = True, sink=None, group=None, source=None) -> ExtractStats:
    """Encode clips [0, n_clips) clip-sharded over `world` ranks (ShardedExtractor.run)."""
    return ShardedExtractor(model, n_clips, n_samples, batch, rank, world, device, gather, sink, group,
                            source).run()


# ------------------------------------------------------------------------------------------------
# the extraction CLI: python -m audiotokenization_amd.extract  (extract_indices.py:375-589)
# ------------------------------------------------------------------------------------------------
VALID_SUBSETS = {"dev-clean", "dev-other", "test-clean", "test-other", "train-clean-100", "train-clean-360",
                 "train-other-500"}


def find_items(root: str, subsets, dataset_path: str = "LibriTTS", ext_audio: str = ".flac"):
    """LibriTTSDataset's walker (extract_indices.py:181-248): per subset, <root>/<dataset_path>/<subset>
    or else <root>/<subset>, every *<ext_audio> below it (rglob) -> [(subset, subset_path, fileid)]."""
    from pathlib import Path

    items = []
    for subset in ([subsets] if isinstance(subsets, str) else subsets):
        if subset not in VALID_SUBSETS:
            print(f"Warning: Subset '{subset}' not in standard {dataset_path} list: {VALID_SUBSETS}")
        subset_path = os.path.join(root, dataset_path, subset)
        if not os.path.isdir(subset_path):
            subset_path = os.path.join(root, subset)
            if not os.path.isdir(subset_path):
                raise RuntimeError(f"Dataset subset not found at expected locations relative to root '{root}': "
                                   f"check structure.")
        for p in sorted(Path(subset_path).rglob(f"*{ext_audio}")):
            items.append((subset, subset_path, p.stem))
    return items


def item_path(subset_path: str, fileid: str, ext_audio: str) -> str:
    """load_libritts_item's path (extract_indices.py:48-72): <subset_path>/<speaker>/<chapter>/<fileid><ext>
    from a LibriTTS (spk_chapter_seg_utt) or LibriSpeech (spk-chapter-utt) file id."""
    parts = fileid.split("_")
    if len(parts) != 4:
        parts = fileid.split("-")
        if len(parts) < 3:
            raise ValueError(f"Cannot parse speaker/chapter from fileid: {fileid}")
    return os.path.join(subset_path, parts[0], parts[1], fileid + ext_audio)


def build_lm(save_path: str, device):
    """extract_indices.py:430-460 + BigCodecModel(ckpt, cfg): hydra/config.yaml and the first existing
    last.ckpt candidate (config.find_checkpoint) -> a CodecLightningModule on `device`."""
    from .config import find_checkpoint, load_config
    from .lightning_shim import CodecLightningModule

    config_path, ckpt_path = find_checkpoint(save_path)
    if not os.path.exists(config_path):
        raise FileNotFoundError(f"Config file not found at {config_path}")
    if ckpt_path is None:
        raise FileNotFoundError(f"Checkpoint file not found under {save_path}")
    return CodecLightningModule.from_checkpoint(ckpt_path, load_config(config_path)).to(device).eval()


def run_extraction(lm, items, output_dir: str, sample_rate: Optional[int], duration: Optional[float],
                   ext_audio: str, device, rank: int = 0, world: int = 1, workers: int = 4, log=print):
    """The extraction loop (extract_indices.py:497-574) for this rank's block of the file list: host decode
    (FLAC / WAV) of the next files on `workers` threads while the current one runs on the GPU, then
    resample (GPU) -> encode -> VQ -> (F, Nq) int16 -> <output_dir>/<subset>/<spk>/<chapter>/<fileid>.npy.
    Per-file failures are counted, not fatal.  Returns (saved, errors) of this rank."""
    from concurrent.futures import ThreadPoolExecutor

    from .ingest import read_audio, load_item

    model = BigCodecModel(lm)
    lo, hi = shard_range(len(items), rank, world)
    mine = items[lo:hi]
    saved = errors = 0

    def read(it):
        subset, subset_path, fileid = it
        path = item_path(subset_path, fileid, ext_audio)
        if not os.path.exists(path):
            raise FileNotFoundError(f"Audio file not found at: {path}")
        return read_audio(path)

    workers = max(1, workers)
    with ThreadPoolExecutor(max_workers=workers) as pool:
        futs = {j: pool.submit(read, mine[j]) for j in range(min(workers, len(mine)))}
        for i, (subset, _, fileid) in enumerate(mine):
            if i + workers < len(mine):  # keep `workers` files decoding ahead of the GPU
                futs[i + workers] = pool.submit(read, mine[i + workers])
            try:
                x, sr = futs.pop(i).result()
                wav, _ = load_item(None, sample_rate, duration, None, device, decoded=(x, sr))
                with torch.no_grad():
                    out = model(wav.unsqueeze(0))
                indices = out.get("indices") if isinstance(out, dict) else None
                if indices is None:
                    log(f"Warning: No indices found for file: {fileid}. Skipping.")
                    errors += 1
                    continue
                save_indices(output_dir, subset, fileid, indices_to_numpy(indices))
                saved += 1
            except Exception as e:  # extract_indices.py:565-574: counted, not fatal
                log(f"Error processing {fileid}: {type(e).__name__}: {e}")
                errors += 1
    return saved, errors


def main(argv=None):
    """python -m audiotokenization_amd.extract --save_path RUN --subsets test-clean [...] — the reference
    CLI's arguments (extract_indices.py:379-389); --workers (host decode threads) is this build's own.
    Under torchrun every rank extracts its block of the file list (clip-sharded, no collective on the
    data path; the saved / error counts are summed at the end)."""
    import argparse
    import sys

    p = argparse.ArgumentParser(description="BigCodec index extraction on MI355X (extract_indices.py)")
    p.add_argument("--dataset_root", type=str, default="../../datasets")
    p.add_argument("--save_path", type=str, required=True, help="run directory with hydra/config.yaml and last.ckpt")
    p.add_argument("--output_folder", type=str, default="extracted_indices")
    p.add_argument("--duration", type=float, default=None)
    p.add_argument("--sample_rate", type=int, default=16000)
    p.add_argument("--dataset_path", type=str, default="LibriTTS")
    p.add_argument("--ext_audio", type=str, default=".flac")
    p.add_argument("--subsets", type=str, nargs="+", required=True)
    p.add_argument("--workers", type=int, default=4)
    a = p.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not os.path.isdir(a.save_path):
        print(f"Error: Model save path does not exist: {a.save_path}")
        return 1
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    output_dir = os.path.join(a.save_path, a.output_folder)
    os.makedirs(output_dir, exist_ok=True)
    lm = build_lm(a.save_path, device)
    items = find_items(a.dataset_root, a.subsets, a.dataset_path, a.ext_audio)
    if not items:
        print("Error: Dataset is empty. Check dataset root, subset names, and file structure.")
        return 1
    if rank == 0:
        print(f"Dataset size: {len(items)} files, {world} rank(s)")
    saved, errors = run_extraction(lm, items, output_dir, a.sample_rate, a.duration, a.ext_audio, device, rank,
                                   world, a.workers)
    if world > 1:
        t = torch.tensor([saved, errors], device=device, dtype=torch.int64)
        dist.all_reduce(t)
        saved, errors = (int(v) for v in t.tolist())
        dist.destroy_process_group()
    if rank == 0:
        print("\nExtraction complete.")
        print(f"Successfully saved {saved} index files.")
        if errors:
            print(f"Encountered {errors} errors.")
        print(f"Indices saved in: {output_dir}")
    sys.stdout.flush()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
