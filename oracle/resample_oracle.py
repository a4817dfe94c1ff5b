"""CPU oracle for the real-audio ingest — TEST INFRASTRUCTURE ONLY (tests/ may import it; the product
never does).

Restates, on torch CPU ops, what the reference runs in extract_indices.py:98-137 (load_libritts_item):
soundfile's float32 WAV read, trim / pad to `duration`, torchaudio.transforms.Resample(orig, new) and
pad_to_stride.  The resampler follows torchaudio's published algorithm (torchaudio/functional/
functional.py: _get_sinc_resample_kernel with resampling_method='sinc_interp_hann', lowpass_filter_width
6, rolloff 0.99, the kernel built in float64 and cast to float32; _apply_sinc_resample_kernel: pad by
(width, width + orig), conv1d(stride=orig), interleave the phases, keep ceil(new * L / orig)).

PARITY UNPINNED: torchaudio and soundfile are not installed in this image and the reference holds no
resampled fixtures, so this restatement cannot be checked against the reference's own output.  It is
checked against an independent evaluation (tests/test_ingest.py: Python's `wave` module for PCM16, a
float64 direct-form sum for the resampler).
"""
from __future__ import annotations

import math
import wave
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F


def read_wav_pcm16(path: str) -> torch.Tensor:
    """soundfile float32 read of a PCM16 WAV via Python's `wave` module: (C, T) = int16 / 32768."""
    with wave.open(path, "rb") as w:
        assert w.getsampwidth() == 2, "oracle reads PCM16 only"
        ch = w.getnchannels()
        raw = w.readframes(w.getnframes())
    x = np.frombuffer(raw, "<i2").astype(np.float32) / np.float32(32768.0)
    return torch.from_numpy(np.ascontiguousarray(x.reshape(-1, ch).T))


def sinc_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    """torchaudio _get_sinc_resample_kernel (sinc_interp_hann): ((new, 1, K) float32, width, orig, new)."""
    g = math.gcd(orig_freq, new_freq)
    orig, new = orig_freq // g, new_freq // g
    base_freq = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base_freq)
    idx = torch.arange(-width, width + orig, dtype=torch.float64)[None, None] / orig
    t = torch.arange(0, -new, -1, dtype=torch.float64)[:, None, None] / new + idx
    t *= base_freq
    t = t.clamp_(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t *= math.pi
    scale = base_freq / orig
    kernels = torch.where(t == 0, torch.tensor(1.0).to(t), t.sin() / t)
    kernels *= window * scale
    return kernels.to(torch.float32), width, orig, new


def resample(x: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """torchaudio.transforms.Resample(orig_freq, new_freq)(x) for float32 x (..., L)."""
    if orig_freq == new_freq:
        return x
    kern, width, orig, new = sinc_kernel(orig_freq, new_freq)
    shape = x.shape
    x = x.reshape(-1, shape[-1])
    n, length = x.shape
    x = F.pad(x, (width, width + orig))
    y = F.conv1d(x[:, None], kern, stride=orig)
    y = y.transpose(1, 2).reshape(n, -1)
    target = int(math.ceil(new * length / orig))
    return y[..., :target].reshape(shape[:-1] + (-1,))


def load_item(path: str, target_sample_rate: Optional[int] = None, duration: Optional[float] = None,
              pad_to_stride: Optional[int] = None, sample_rate: int = 16000):
    """extract_indices.py:36-140 with offset_mode='start' for a PCM16 WAV of `sample_rate`."""
    x = read_wav_pcm16(path)
    sr = sample_rate
    if duration is not None:
        n = int(duration * sr)
        if x.size(1) < n:
            x = F.pad(x, (0, n - x.size(1)))
        x = x[:, :n]
    if target_sample_rate and target_sample_rate != sr:
        x = resample(x.float(), sr, target_sample_rate)
        sr = target_sample_rate
    if pad_to_stride and x.size(1) % pad_to_stride != 0:
        x = F.pad(x, (0, pad_to_stride - x.size(1) % pad_to_stride))
    return x, sr
