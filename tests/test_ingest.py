"""Real-audio ingest (audiotokenization_amd/ingest.py, csrc/resample.hip).

Oracle: oracle/resample_oracle.py, a torch-CPU restatement of torchaudio's Resample and soundfile's read.
Parity is UNPINNED against the reference itself (torchaudio / soundfile are absent from this image); the
oracle is checked here against independent float64 / `wave`-module evaluations instead.

Tolerances: WAV decoding bit-exact; sinc filters equal to the float32 cast of the float64 design within
1 ulp; resampled samples max|d| / max|ref| <= 2e-6 (fp32 sums of 16-171 taps in a different order than
oneDNN's conv); encoder latents 1e-4 and VQ indices equal except certified near-ties (test_gpu_model.py).
"""
import math
import os
import struct
import wave

import numpy as np
import pytest
import torch

from audiotokenization_amd import ingest
from oracle import resample_oracle as RO

RATES = [(16000, 24000), (44100, 24000), (24000, 16000), (22050, 24000), (8000, 24000), (48000, 24000)]
REF_WAVS = "/root/reference/BigCodec_SSL/speaker_verification/vox1_data"


def _write_riff(path, tag, channels, rate, bits, payload: bytes):
    align = channels * bits // 8
    fmt = struct.pack("<HHIIHH", tag, channels, rate, rate * align, align, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(payload)) + payload
    if len(payload) & 1:
        body += b"\0"
    with open(path, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def _pcm16_file(path, x16: np.ndarray, rate=16000, channels=1):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(x16.astype("<i2").tobytes())


def test_read_wav_formats(tmp_path):
    rng = np.random.default_rng(0)
    v16 = rng.integers(-32768, 32768, size=(500, 2)).astype(np.int16)
    _pcm16_file(tmp_path / "a.wav", v16.reshape(-1), channels=2)
    x, sr = ingest.read_wav(str(tmp_path / "a.wav"))
    assert sr == 16000 and x.shape == (2, 500) and x.dtype == np.float32
    assert np.array_equal(x, v16.T.astype(np.float32) / 32768.0)
    v8 = rng.integers(0, 256, size=300).astype(np.uint8)
    _write_riff(tmp_path / "b.wav", 1, 1, 8000, 8, v8.tobytes())
    x, sr = ingest.read_wav(str(tmp_path / "b.wav"))
    assert sr == 8000 and np.array_equal(x[0], (v8.astype(np.float32) - 128) / 128)
    v24 = rng.integers(-(1 << 23), 1 << 23, size=301)
    b24 = b"".join(int(v & 0xFFFFFF).to_bytes(3, "little") for v in v24)
    _write_riff(tmp_path / "c.wav", 1, 1, 24000, 24, b24)
    x, _ = ingest.read_wav(str(tmp_path / "c.wav"))
    assert np.array_equal(x[0], v24.astype(np.float32) / 8388608.0)
    v32 = rng.integers(-(1 << 31), 1 << 31, size=64).astype(np.int32)
    _write_riff(tmp_path / "d.wav", 1, 1, 24000, 32, v32.astype("<i4").tobytes())
    x, _ = ingest.read_wav(str(tmp_path / "d.wav"))
    assert np.array_equal(x[0], v32.astype(np.float32) * np.float32(2.0 ** -31))
    f32 = rng.standard_normal(77).astype(np.float32)
    _write_riff(tmp_path / "e.wav", 3, 1, 44100, 32, f32.astype("<f4").tobytes())
    x, sr = ingest.read_wav(str(tmp_path / "e.wav"))
    assert sr == 44100 and np.array_equal(x[0], f32)
    (tmp_path / "f.flac").write_bytes(b"fLaC\0\0\0\0")
    with pytest.raises(ValueError):  # FLAC goes to the FLAC decoder (tests/test_flac.py), which rejects this stub
        ingest.read_wav(str(tmp_path / "f.flac"))


@pytest.mark.skipif(not os.path.isdir(REF_WAVS), reason="reference data not present (GPU box)")
def test_read_reference_wavs_like_wave_module():
    """The reference's own recordings (VoxCeleb excerpts it ships, 16 kHz PCM16) decode like `wave` / 32768."""
    n = 0
    for root, _, files in os.walk(REF_WAVS):
        for f in sorted(files):
            if f.endswith(".wav"):
                p = os.path.join(root, f)
                x, sr = ingest.read_wav(p)
                assert sr == 16000
                assert torch.equal(torch.from_numpy(x), RO.read_wav_pcm16(p))
                n += 1
    assert n >= 1


@pytest.mark.parametrize("orig,new", RATES)
def test_sinc_filters_match_oracle_design(orig, new):
    k, width, o, nw = ingest.sinc_resample_kernel(orig, new)
    kr, wr, orr, nr = RO.sinc_kernel(orig, new)
    assert (width, o, nw) == (wr, orr, nr) and k.shape == (nw, 2 * width + o)
    a, b = torch.from_numpy(k), kr[:, 0]
    ulp = torch.nextafter(b.abs(), torch.tensor(float("inf"))) - b.abs()
    assert bool(((a - b).abs() <= ulp).all())


@pytest.mark.parametrize("orig,new", RATES[:3])
def test_oracle_resampler_against_direct_float64(orig, new):
    """The oracle's conv1d formulation against a direct float64 sum of the same filters."""
    x = torch.from_numpy(np.random.default_rng(orig + new).standard_normal((2, 913)).astype(np.float32))
    y = RO.resample(x, orig, new)
    k, width, o, nw = ingest.sinc_resample_kernel(orig, new)
    n = x.shape[1]
    lout = math.ceil(nw * n / o)
    xp = np.pad(x.double().numpy(), ((0, 0), (width, width + o)))
    ref = np.zeros((2, lout))
    for j in range(lout):
        jj, kk = divmod(j, nw)
        ref[:, j] = xp[:, jj * o: jj * o + k.shape[1]] @ k[kk].astype(np.float64)
    assert y.shape == (2, lout)
    assert float(np.abs(y.double().numpy() - ref).max() / np.abs(ref).max()) < 1e-6


def test_oracle_resampler_passes_a_low_tone():
    t = np.arange(16000) / 16000.0
    x = torch.from_numpy(np.sin(2 * np.pi * 440 * t).astype(np.float32))[None]
    y = RO.resample(x, 16000, 24000)[0].double().numpy()
    ref = np.sin(2 * np.pi * 440 * np.arange(24000) / 24000.0)
    assert y.shape == (24000,)
    assert np.abs(y[600:-600] - ref[600:-600]).max() < 2e-3


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("orig,new", RATES)
@pytest.mark.parametrize("n", [1, 5, 3001, 16001])
def test_gpu_resampler_matches_oracle(dev, orig, new, n):
    x = torch.from_numpy(np.random.default_rng(n + orig).standard_normal((3, n)).astype(np.float32))
    ref = RO.resample(x, orig, new)
    y = ingest.Resampler.get(orig, new, dev)(x.to(dev)).cpu()
    assert y.shape == ref.shape
    err = float((y - ref).abs().max() / ref.abs().max().clamp_min(1e-30))
    assert err <= 2e-6, err


@pytest.mark.gpu
@pytest.mark.parametrize("duration,stride", [(None, 200), (0.9, None), (1.7, 200)])
def test_gpu_load_item_then_encode_matches_oracle(dev, tmp_path, duration, stride):
    """A 16 kHz PCM16 WAV through load_item (read -> trim/pad -> GPU resample -> pad to stride) and the
    encoder + VQ, against the oracle's load_libritts_item restatement and CPU encoder."""
    from helpers import assert_close_rel, build_models, index_mismatches, top2_gap, torch_sd
    from oracle import bigcodec_oracle as O

    rng = np.random.default_rng(11)
    t = np.arange(int(1.3 * 16000)) / 16000.0
    sig = 0.4 * np.sin(2 * np.pi * (200 + 900 * t) * t) + 0.05 * rng.standard_normal(t.size)
    path = tmp_path / "utt.wav"
    _pcm16_file(path, np.clip(np.round(sig * 32767), -32768, 32767))
    x, sr = ingest.load_item(str(path), 24000, duration=duration, pad_to_stride=stride, device=dev)
    xr, srr = RO.load_item(str(path), 24000, duration=duration, pad_to_stride=stride)
    assert sr == srr == 24000 and tuple(x.shape) == tuple(xr.shape)
    assert float((x.cpu() - xr).abs().max()) <= 2e-6 * float(xr.abs().max())
    enc, dec, esd, dsd, ek, _ = build_models("debug", device=dev)
    with torch.no_grad():
        lat = enc(x[None])
        codes = dec(lat, vq=True)[1].cpu()
        lat_ref = O.encoder_forward(xr[None], torch_sd(esd), ek)
        _, codes_ref, _ = O.rvq_forward(lat_ref, torch_sd(dsd))
        _, _, _, ze_ref = O.fvq_forward(lat_ref, torch_sd(dsd), "quantizer.layers.0.", return_ze=True)
    assert_close_rel(lat.cpu(), lat_ref, 1e-4, "latent of ingested audio")
    gap = top2_gap(ze_ref, torch.from_numpy(dsd["quantizer.layers.0._codebook.weight"]))
    n_bad, worst = index_mismatches(codes.numpy(), codes_ref.numpy(), gap)
    print(f"ingest duration={duration} stride={stride}: {n_bad} / {codes.numel()} index mismatches")
