"""Real-audio ingest for index extraction.

The reference loads each utterance with soundfile, trims / zero-pads it to `duration`, resamples it with
torchaudio.transforms.Resample and pads it to a stride (extract_indices.py:36-140, load_libritts_item;
data_module.py:95-98 does the same resampling for training).  Here:

  * Decoding runs on the host: `read_wav` (RIFF/WAVE PCM 8/16/24/32-bit and IEEE float) and `read_flac`
    (the library's from-scratch RFC 9639 decoder, csrc/flac.cpp: the reference's actual input format),
    both scaled the way soundfile's float32 reads scale them; `read_audio` picks by the file's magic.
  * Resampling runs on the GPU (`bc_resample_sinc`, csrc/resample.hip) with the sinc-Hann filters built
    here exactly as torchaudio builds them (`sinc_resample_kernel`, float64 -> float32).
  * `load_item` restates load_libritts_item's order of operations for offset_mode='start' (the mode
    extract_indices.py:473 uses): read -> trim/pad to duration -> resample -> pad to stride.

torchaudio is absent from this image, so the resampler's parity is pinned only against the restatement in
oracle/resample_oracle.py (its published algorithm); see DESIGN.md.
"""
from __future__ import annotations

import math
import struct
from ctypes import byref as ctypes_ref
from ctypes import c_int as ctypes_int
from ctypes import c_longlong as ctypes_longlong
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib as L
from . import ops


def read_wav(path: str) -> Tuple[np.ndarray, int]:
    """(waveform (C, T) float32, sample_rate) of a RIFF/WAVE file, as
    soundfile.SoundFile(path).read(dtype='float32', always_2d=True).T gives it (extract_indices.py:98-106):
    PCM is divided by 2^(bits - 1) (8-bit PCM is unsigned: (v - 128) / 128), IEEE float is read as is."""
    with open(path, "rb") as fh:
        data = fh.read()
    if data[:4] == b"fLaC":
        return read_flac(path, data)
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    fmt = pcm = None
    pos = 12
    while pos + 8 <= len(data):
        cid = data[pos:pos + 4]
        size = struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = body
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None or len(fmt) < 16:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, channels, rate, _, align, bits = struct.unpack("<HHIIHH", fmt[:16])
    if tag == 0xFFFE and len(fmt) >= 26:  # WAVE_FORMAT_EXTENSIBLE: the sub-format's first two bytes
        tag = struct.unpack("<H", fmt[24:26])[0]
    if channels < 1 or align != channels * ((bits + 7) // 8):
        raise ValueError(f"{path}: inconsistent fmt chunk")
    n = len(pcm) // align
    raw = pcm[: n * align]
    if tag == 1 and bits == 8:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif tag == 1 and bits == 16:
        x = np.frombuffer(raw, "<i2").astype(np.float32) / np.float32(32768.0)
    elif tag == 1 and bits == 24:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        x = ((v ^ 0x800000) - 0x800000).astype(np.float32) / np.float32(8388608.0)
    elif tag == 1 and bits == 32:
        x = np.frombuffer(raw, "<i4").astype(np.float32) * np.float32(2.0 ** -31)
    elif tag == 3 and bits == 32:
        x = np.frombuffer(raw, "<f4").astype(np.float32)
    elif tag == 3 and bits == 64:
        x = np.frombuffer(raw, "<f8").astype(np.float32)
    else:
        raise NotImplementedError(f"{path}: WAV format tag {tag} with {bits} bits")
    return np.ascontiguousarray(x.reshape(n, channels).T), int(rate)


_FLAC_ERR = {1: "bad argument", 2: "not a FLAC stream or corrupt", 3: "unsupported FLAC feature",
             4: "CRC mismatch", 5: "more samples than STREAMINFO announced"}


def read_flac(path: str, data: bytes = None, check_crc: bool = True, as_int: bool = False) -> Tuple[np.ndarray, int]:
    """(waveform (C, T), sample_rate) of a FLAC file through bc_flac_decode (host decoder in
    libbigcodec_hip.so): float32 = sample / 2^(bits - 1) as soundfile.SoundFile(path).read(dtype='float32',
    always_2d=True).T gives it (extract_indices.py:98-106); as_int -> the int32 samples."""
    if data is None:
        with open(path, "rb") as fh:
            data = fh.read()
    lib = L.load()
    buf = np.frombuffer(data, dtype=np.uint8)
    rate, ch, bits, total = (ctypes_int(), ctypes_int(), ctypes_int(), ctypes_longlong())
    rc = lib.bc_flac_info(buf.ctypes.data, len(data), ctypes_ref(rate), ctypes_ref(ch), ctypes_ref(bits),
                          ctypes_ref(total))
    if rc:
        raise ValueError(f"{path}: {_FLAC_ERR.get(rc, rc)}")
    cap = int(total.value) if total.value > 0 else max(4096, len(data))
    while True:
        out = np.empty((ch.value, cap), dtype=np.int32 if as_int else np.float32)
        n = lib.bc_flac_decode(buf.ctypes.data, len(data), out.ctypes.data, int(as_int), cap, int(check_crc))
        if n == -5 and total.value <= 0:  # unknown length: grow and decode again
            cap *= 4
            continue
        if n < 0:
            raise ValueError(f"{path}: {_FLAC_ERR.get(-n, n)}")
        return np.ascontiguousarray(out[:, :n]), int(rate.value)


def read_audio(path: str) -> Tuple[np.ndarray, int]:
    """WAV or FLAC by content (soundfile's float32 read for either)."""
    return read_wav(path)


def sinc_resample_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6,
                         rolloff: float = 0.99) -> Tuple[np.ndarray, int, int, int]:
    """torchaudio.functional._get_sinc_resample_kernel (resampling_method='sinc_interp_hann', the
    default of transforms.Resample) restated: returns (filters (new, K) float32, width, orig, new) with
    orig / new divided by their gcd and K = 2 * width + orig.  Built in float64, cast to float32."""
    if orig_freq <= 0 or new_freq <= 0:
        raise ValueError("sample rates must be positive")
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base_freq = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base_freq)
    idx = np.arange(-width, width + orig, dtype=np.float64)[None, :] / orig
    t = np.arange(0, -new, -1, dtype=np.float64)[:, None] / new + idx
    t = t * base_freq
    t = np.clip(t, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    scale = base_freq / orig
    with np.errstate(invalid="ignore", divide="ignore"):
        kernels = np.where(t == 0, 1.0, np.sin(t) / t)
    kernels = kernels * (window * scale)
    return kernels.astype(np.float32), width, orig, new


class Resampler:
    """transforms.Resample(orig_freq, new_freq) on the GPU: (..., L) float32 device tensor ->
    (..., ceil(new * L / orig)); identity when the rates are equal (as torchaudio returns its input)."""

    _cache: Dict[Tuple[int, int, str], "Resampler"] = {}

    def __init__(self, orig_freq: int, new_freq: int, device):
        self.orig_freq, self.new_freq = int(orig_freq), int(new_freq)
        kern, self.width, self.orig, self.new = sinc_resample_kernel(self.orig_freq, self.new_freq)
        self.taps = kern.shape[1]
        self.kern = torch.from_numpy(kern).to(device)

    @classmethod
    def get(cls, orig_freq: int, new_freq: int, device) -> "Resampler":
        key = (int(orig_freq), int(new_freq), str(torch.device(device)))
        if key not in cls._cache:
            cls._cache[key] = cls(orig_freq, new_freq, device)
        return cls._cache[key]

    def out_len(self, n: int) -> int:
        return -(-self.new * n // self.orig)

    def __call__(self, x: torch.Tensor, pad_to: int = 0) -> torch.Tensor:
        if self.orig_freq == self.new_freq:
            return x
        if not x.is_cuda or x.dtype != torch.float32:
            raise L.BigCodecLibraryError("Resampler takes float32 device tensors")
        x = x.contiguous()
        lout = self.out_len(int(x.shape[-1]))
        pitch = max(lout, pad_to)
        return ops.load().resample_sinc(x, self.kern, lout, pitch, self.orig, self.new, self.taps, self.width)


def load_item(path: str, target_sample_rate: Optional[int] = None, duration: Optional[float] = None,
              pad_to_stride: Optional[int] = None, device="cuda",
              decoded: Optional[Tuple[np.ndarray, int]] = None) -> Tuple[torch.Tensor, int]:
    """extract_indices.py:36-140 (offset_mode='start') for one file: (waveform (C, T) on `device`,
    sample rate).  Trim / zero-pad at the end to int(duration * sr) samples, resample on the GPU,
    zero-pad at the end to a multiple of pad_to_stride."""
    x, sr = decoded if decoded is not None else read_audio(path)
    if duration is not None:
        n = int(duration * sr)
        x = x[:, :n] if x.shape[1] >= n else np.pad(x, ((0, 0), (0, n - x.shape[1])))
    t = torch.from_numpy(np.ascontiguousarray(x))
    if torch.device(device).type == "cuda":
        t = t.pin_memory().to(device, non_blocking=True)
    if target_sample_rate and target_sample_rate != sr:
        rs = Resampler.get(sr, target_sample_rate, t.device)
        lout = rs.out_len(t.shape[1])
        pad = lout if not pad_to_stride or lout % pad_to_stride == 0 else lout + pad_to_stride - lout % pad_to_stride
        return rs(t, pad_to=pad), int(target_sample_rate)
    if pad_to_stride and t.shape[1] % pad_to_stride:
        t = torch.nn.functional.pad(t, (0, pad_to_stride - t.shape[1] % pad_to_stride))
    return t, sr
