"""Deterministic synthetic weights and white-noise clips.

No trained checkpoint exists for the reference, so parity and benchmarks run on weights synthesised
from a counter hash.  The same spec is applied to the reference modules by tools/make_golden.py, so
both sides load bit-identical parameters.

Weight spec (per state_dict entry, keyed by its name):
  u(name, i)   = (splitmix64(fnv1a64(name) ^ (seed * 0x9E3779B97F4A7C15) + i) >> 40) * 2^-24
  *.weight_v / *.weight (conv, linear)   uniform(-1/sqrt(fan_in), 1/sqrt(fan_in)), fan_in = prod(shape[1:])
  *.weight_g                             ||v|| (per dim-0 slice) * uniform(0.75, 1.25)
  *.bias (conv, linear)                  uniform(-1/sqrt(fan_in), +) with the sibling weight's fan_in
  LSTM weight_* / bias_*                 uniform(-1/sqrt(H), 1/sqrt(H))      (torch's own init range)
  *.alpha / *.beta (Snake, log scale)    uniform(-0.5, 0.5)
  *._codebook.weight                     uniform(-1, 1)
  *.filter (anti-alias buffers)          left as constructed (deterministic Kaiser-sinc)
Clip spec: x[i, n] = (splitmix64(0xB16C0DEC ^ (i << 32) ^ n) >> 40) * 2^-24 - 0.5   (exact fp32)
"""
from __future__ import annotations

import re
from typing import Dict, Mapping

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for ch in s.encode():
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def hash_uniform01(name: str, n: int, seed: int = 0) -> np.ndarray:
    """n values in [0, 1) with 24-bit resolution (exactly representable in fp32)."""
    key = (fnv1a64(name) ^ ((seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = splitmix64(np.uint64(key) + idx)
    return (h >> np.uint64(40)).astype(np.float64) * (1.0 / (1 << 24))


def _uniform(name: str, shape, lo: float, hi: float, seed: int) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = hash_uniform01(name, n, seed)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


_LSTM_RE = re.compile(r"\.(weight_ih|weight_hh|bias_ih|bias_hh)_l\d+(_reverse)?$")


def synth_state_dict(template: Mapping[str, "np.ndarray | object"], seed: int = 0) -> Dict[str, np.ndarray]:
    """Return {name: float32 ndarray} for every entry of `template` (name -> tensor/array/shape).

    Anti-alias filter buffers are copied from the template unchanged."""
    shapes = {}
    for k, v in template.items():
        shapes[k] = tuple(v.shape) if hasattr(v, "shape") else tuple(v)
    out: Dict[str, np.ndarray] = {}
    # pass 1: weights (v first so g can use ||v||)
    for k, shp in shapes.items():
        if k.endswith(".filter"):
            v = template[k]
            arr = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
            out[k] = arr.astype(np.float32).copy()
        elif _LSTM_RE.search(k):
            # hidden size = rows/4 for weight_*, len/4 for bias_*
            hid = shp[0] // 4
            b = 1.0 / np.sqrt(hid)
            out[k] = _uniform(k, shp, -b, b, seed)
        elif k.endswith("._codebook.weight"):
            out[k] = _uniform(k, shp, -1.0, 1.0, seed)
        elif k.endswith(".alpha") or k.endswith(".beta"):
            out[k] = _uniform(k, shp, -0.5, 0.5, seed)
        elif k.endswith(".weight_v") or (k.endswith(".weight") and len(shp) >= 2):
            fan_in = int(np.prod(shp[1:]))
            b = 1.0 / np.sqrt(fan_in)
            out[k] = _uniform(k, shp, -b, b, seed)
    for k, shp in shapes.items():
        if k in out:
            continue
        if k.endswith(".weight_g"):
            v = out[k[: -len("weight_g")] + "weight_v"].astype(np.float64)
            nrm = np.sqrt((v.reshape(v.shape[0], -1) ** 2).sum(1))
            scale = _uniform(k, (shp[0],), 0.75, 1.25, seed).astype(np.float64)
            out[k] = (nrm * scale).astype(np.float32).reshape(shp)
        elif k.endswith(".bias"):
            prefix = k[: -len("bias")]
            sib = prefix + "weight_v" if (prefix + "weight_v") in shapes else prefix + "weight"
            if sib in shapes:
                fan_in = int(np.prod(shapes[sib][1:]))
            else:
                fan_in = shp[0]
            b = 1.0 / np.sqrt(fan_in)
            out[k] = _uniform(k, shp, -b, b, seed)
        else:
            raise KeyError(f"synth_state_dict: no rule for parameter {k!r} {shp}")
    return out


def synth_clips(n_clips: int, n_samples: int, clip0: int = 0) -> np.ndarray:
    """(n_clips, n_samples) float32 white noise in [-0.5, 0.5)."""
    i = (np.arange(n_clips, dtype=np.uint64) + np.uint64(clip0))[:, None]
    n = np.arange(n_samples, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        h = splitmix64(np.uint64(0xB16C0DEC) ^ (i << np.uint64(32)) ^ n)
    u = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))
    return (u - np.float32(0.5)).astype(np.float32)
