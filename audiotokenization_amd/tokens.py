"""Token -> audio service path: the other half of the tokenizer.

Consumes the index files the extraction path writes (extract_indices.py:512-561 format, restated in
extract.py: one `.npy` per clip, int16, shape (F, Nq)), batches them, and decodes them on the GPU:

    codes (B, F, Nq) int64  --bc_vq2emb_ct-->  emb (B, D, F)  --BigCodecDecoder.decode-->  wav (B, 1, F * hop)

which is the reference's `decoder.vq2emb(codes)` (codec_decoder.py:96-99 -> residual_vq.py:42-48 ->
factorized_vector_quantize.py:78-81), the caller's `.transpose(1, 2)`, then `decoder(x, vq=False)`
(codec_decoder.py:85-94).  Host work is limited to reading the files, validating the indices (an index
outside the codebook raises here; on the device it would decode to NaN) and one pinned upload per batch.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence, Tuple

import numpy as np
import torch


def load_indices(path: str) -> np.ndarray:
    """One clip's index file (extract.save_indices): int16 (F, Nq) -> the same array, validated."""
    arr = np.load(path, allow_pickle=False)
    if arr.ndim == 1:  # a single-quantizer file written as (F,)
        arr = arr[:, None]
    if arr.ndim != 2 or arr.dtype.kind not in "iu":
        raise ValueError(f"{path}: expected an integer (F, Nq) index array, got {arr.dtype} {arr.shape}")
    return arr


def codes_to_device(arrs: Sequence[np.ndarray], device, n_codes: int) -> Tuple[torch.Tensor, List[int]]:
    """Stack (F_i, Nq) index arrays into one (B, F_max, Nq) int64 device tensor (ragged clips padded
    with code 0 and cut again by `decode_codes`; the padding changes a shorter clip's last frames through
    the decoder's receptive field, so `decode_index_files` batches equal lengths only).  int16 files store codes
    >= 32768 as negatives (extract_indices.py:540 `astype(np.int16)`), so they are read back modulo
    2^16 before the range check."""
    if not arrs:
        raise ValueError("no index arrays")
    nq = {a.shape[1] for a in arrs}
    if len(nq) != 1:
        raise ValueError(f"mixed quantizer counts {sorted(nq)} in one batch")
    lengths = [int(a.shape[0]) for a in arrs]
    host = np.zeros((len(arrs), max(lengths), nq.pop()), dtype=np.int64)
    for i, a in enumerate(arrs):
        v = a.astype(np.int64)
        if a.dtype == np.int16:
            v = v & 0xFFFF
        if v.size and (v.min() < 0 or v.max() >= n_codes):
            raise ValueError(f"clip {i}: index outside [0, {n_codes})")
        host[i, : a.shape[0]] = v
    t = torch.from_numpy(host)
    if torch.device(device).type == "cuda":
        t = t.pin_memory().to(device, non_blocking=True)
    return t, lengths


def decode_codes(decoder, codes: torch.Tensor, lengths: Sequence[int] | None = None) -> List[torch.Tensor]:
    """codes (B, F, Nq) int64 on the device -> per-clip waveforms (1, F_i * hop) on the device."""
    with torch.no_grad():
        wav = decoder.tokens_to_audio(codes)
    hop = int(decoder.hop_length)
    lengths = lengths if lengths is not None else [codes.shape[1]] * codes.shape[0]
    return [wav[i, :, : n * hop] for i, n in enumerate(lengths)]


def decode_index_files(decoder, paths: Iterable[str], device, batch: int = 16) -> List[np.ndarray]:
    """Decode index files, `batch` clips per launch sequence; returns one float32 (F * hop,) array per
    file, in order.  Clips are batched only with clips of the same length: padding a shorter clip would
    change its last frames through the decoder's receptive field, and the reference decodes each file
    on its own."""
    paths = list(paths)
    q = decoder.quantizer
    n_codes = q.codebook_size if getattr(decoder, "fsq", False) else q.layers[0].codebook_size
    arrs = [load_indices(p) for p in paths]
    groups: dict = {}
    for i, a in enumerate(arrs):
        groups.setdefault(a.shape, []).append(i)
    out: List[np.ndarray] = [None] * len(arrs)  # type: ignore[list-item]
    for idxs in groups.values():
        for lo in range(0, len(idxs), batch):
            part = idxs[lo: lo + batch]
            codes, lengths = codes_to_device([arrs[i] for i in part], device, n_codes)
            for i, w in zip(part, decode_codes(decoder, codes, lengths)):
                out[i] = w[0].cpu().numpy()
    return out
