"""Host FLAC decoder (csrc/flac.cpp, bc_flac_decode) — the reference's input format (extract_indices.py:
98-106 reads LibriTTS / LibriSpeech .flac through soundfile).  No FLAC file, encoder or decoder exists in
this image or the reference, so every case is a lossless round trip through tests/flac_writer.py (an
independent RFC 9639 encoder that forces each feature): the decoded integers must equal the encoded ones
exactly, and the float32 read must equal int / 2^(bits - 1) (libsndfile's normalised read).  Parity with
libFLAC itself is unpinned.  CPU only (host code)."""
import numpy as np
import pytest

from audiotokenization_amd import _lib as L
from audiotokenization_amd import ingest
import flac_writer
from flac_writer import encode


def _signal(C, T, bps, seed, kind="speechy"):
    rng = np.random.default_rng(seed)
    lim = (1 << (bps - 1)) - 1
    if kind == "noise":
        x = rng.integers(-lim - 1, lim + 1, size=(C, T))
    else:  # smooth (predictable) + noise: exercises the predictors' residuals
        t = np.arange(T)
        base = np.sin(2 * np.pi * t * (0.013 + 0.004 * np.arange(C)[:, None])) * 0.6 * lim
        x = base + rng.normal(0, lim * 0.01, size=(C, T))
    return np.clip(np.round(x), -lim - 1, lim).astype(np.int64)


def _decode(data, as_int=True, check_crc=True, cap=None):
    lib = L.load()
    buf = np.frombuffer(data, np.uint8)
    rate, ch, bits, total = (ingest.ctypes_int(), ingest.ctypes_int(), ingest.ctypes_int(), ingest.ctypes_longlong())
    assert lib.bc_flac_info(buf.ctypes.data, len(data), ingest.ctypes_ref(rate), ingest.ctypes_ref(ch),
                            ingest.ctypes_ref(bits), ingest.ctypes_ref(total)) == 0
    cap = cap or max(int(total.value), 1)
    out = np.zeros((ch.value, cap), np.int32 if as_int else np.float32)
    n = lib.bc_flac_decode(buf.ctypes.data, len(data), out.ctypes.data, int(as_int), cap, int(check_crc))
    return n, out, rate.value, bits.value


KINDS = [dict(kind="verbatim")] + [dict(kind="fixed", order=o) for o in range(5)] + \
        [dict(kind="lpc", order=o, lpc_prec=p) for o, p in ((1, 12), (2, 15), (8, 12), (12, 14), (32, 10))]


@pytest.mark.parametrize("bps", [8, 16, 24])
@pytest.mark.parametrize("C", [1, 2])
def test_roundtrip_every_subframe_type(C, bps):
    T = 30000
    x = _signal(C, T, bps, seed=bps * 10 + C)
    plan_kinds = KINDS + [dict(kind="constant")]
    starts = np.cumsum([0] + [1152, 576, 4096, 192, 300, 4608, 1000] * 5)
    for fi in range(len(starts) - 1):  # constant blocks where the plan asks for CONSTANT subframes
        if any((fi * C + c) % len(plan_kinds) == len(plan_kinds) - 1 for c in range(C)):
            x[:, starts[fi]:starts[fi + 1]] = 7 - fi
    flac_writer.EMITTED.clear()

    def plan(fi, c):
        if fi == "stereo":
            return (1, 8, 9, 10)[c % 4]
        k = dict(plan_kinds[(fi * C + c) % len(plan_kinds)])
        k.update(porder=fi % 5, method=(fi + c) % 2, escape_parts=(1,) if fi % 3 == 0 else ())
        return k

    data = encode(x, 16000, bps, block_sizes=[1152, 576, 4096, 192, 300, 4608, 1000], plan=plan)
    n, out, rate, bits = _decode(data)
    assert (n, rate, bits) == (T, 16000, bps)
    np.testing.assert_array_equal(out.astype(np.int64), x)
    f, sr = ingest.read_flac("mem", data)
    assert sr == 16000 and f.dtype == np.float32 and f.shape == (C, T)
    np.testing.assert_array_equal(f, (x.astype(np.float64) / 2 ** (bps - 1)).astype(np.float32))
    kinds = {(k, o) for k, o, *_ in flac_writer.EMITTED}
    assert {("verbatim", 0), ("constant", 0)} | {("fixed", o) for o in range(5)} <= kinds, kinds
    assert {("lpc", o) for o in (1, 2, 8, 12, 32)} <= kinds, kinds
    assert any(e[2] for e in flac_writer.EMITTED) and {e[3] for e in flac_writer.EMITTED if e[0] == "lpc"} == {0, 1}


@pytest.mark.parametrize("assign", [1, 8, 9, 10])
def test_stereo_decorrelation_and_wasted_bits(assign):
    x = _signal(2, 5000, 16, seed=assign, kind="noise") // 8 * 8  # 3 wasted bits in every channel
    x[1] = np.clip(x[1] // 2 + x[0] // 2, -32768, 32760) // 8 * 8

    def plan(fi, c):
        if fi == "stereo":
            return assign
        return dict(kind=("fixed", "lpc", "verbatim")[fi % 3], order=(2, 6, 0)[fi % 3], wasted=3, porder=2)

    n, out, _, _ = _decode(encode(x, 44100, 16, block_sizes=[1024], plan=plan))
    assert n == 5000
    np.testing.assert_array_equal(out.astype(np.int64), x)


def test_header_codes_variable_blocks_and_unknown_length():
    """Sample-rate codes 12 / 13 / 0 (STREAMINFO), sample size 0 (STREAMINFO), variable block sizes (coded
    sample numbers up to several bytes), no extra metadata, total length unknown."""
    x = _signal(1, 70001, 16, seed=3)
    for rate, kw in ((12000, {}), (12345, {}), (16000, dict(rate_in_header=False, size_in_header=False))):
        data = encode(x, rate, 16, block_sizes=[4096, 333, 16384, 192], variable=True, extra_meta=False,
                      total_known=False, **kw)
        f, sr = ingest.read_flac("mem", data, as_int=True)
        assert sr == rate
        np.testing.assert_array_equal(f[0].astype(np.int64), x[0])


def test_corruption_is_detected():
    x = _signal(1, 3000, 16, seed=5)
    data = bytearray(encode(x, 16000, 16, block_sizes=[1024]))
    first = data.index(b"\xff\xf8")
    for off, want in ((first + 5, -4), (len(data) - 40, -4)):
        bad = bytearray(data)
        bad[off] ^= 0x10
        n, _, _, _ = _decode(bytes(bad))
        assert n in (want, -2), n  # CRC mismatch (or a corrupt field found first)
    n, _, _, _ = _decode(bytes(data[: len(data) - 100]))
    assert n < 0  # truncated stream
    n, _, _, _ = _decode(bytes(data), cap=100)
    assert n == -5  # output too small
    with pytest.raises(ValueError):
        ingest.read_flac("mem", b"fLaC\x00\x00")


def test_read_audio_dispatches_on_content(tmp_path):
    x = _signal(1, 2000, 16, seed=9)
    p = tmp_path / "a_0_0_0.flac"
    p.write_bytes(encode(x, 24000, 16, block_sizes=[4096]))
    y, sr = ingest.read_audio(str(p))
    assert sr == 24000
    np.testing.assert_array_equal(y[0], (x[0] / 32768.0).astype(np.float32))
