"""A small FLAC ENCODER written from RFC 9639 for the decoder tests (test infrastructure only).

No FLAC encoder, decoder or .flac file exists in this image or in /root/reference, so the decoder
(audiotokenization_amd/csrc/flac.cpp) is checked by lossless round trips through this independent writer,
which can force every feature the format has: CONSTANT / VERBATIM / FIXED 0-4 / LPC subframes, Rice and
escaped partitions with 4- or 5-bit parameters and partition orders 0-8, wasted bits, the four channel
assignments, fixed and variable block sizes (block-size codes 1-15), sample-rate and sample-size codes,
extra metadata blocks before the frames.  Parity against libFLAC itself stays unpinned (absent).
"""
from __future__ import annotations

import struct
from typing import List, Optional, Sequence

import numpy as np

EMITTED = set()  # (kind, order, escape used, method) of every subframe written: tests check their coverage


class BitWriter:
    def __init__(self):
        self.acc = 0
        self.n = 0

    def u(self, v: int, n: int):
        if n:
            assert 0 <= v < (1 << n), (v, n)
            self.acc = (self.acc << n) | v
            self.n += n

    def s(self, v: int, n: int):
        if n:
            assert -(1 << (n - 1)) <= v < (1 << (n - 1)), (v, n)
            self.u(v & ((1 << n) - 1), n)

    def unary(self, q: int):
        self.u(1, q + 1)  # q zeros then a one

    def align(self):
        if self.n % 8:
            self.u(0, 8 - self.n % 8)

    def bytes(self) -> bytes:
        assert self.n % 8 == 0
        return self.acc.to_bytes(self.n // 8, "big") if self.n else b""


def crc8(data: bytes) -> int:
    c = 0
    for x in data:
        c ^= x
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data: bytes) -> int:
    c = 0
    for x in data:
        c ^= x << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def utf8_number(v: int) -> bytes:
    if v < 0x80:
        return bytes([v])
    for nb, lead in ((2, 0xC0), (3, 0xE0), (4, 0xF0), (5, 0xF8), (6, 0xFC), (7, 0xFE)):
        bits = 5 * 1 + 6 * (nb - 1) if nb == 2 else (7 - nb) + 6 * (nb - 1)
        if nb == 7:
            bits = 36
        if v < (1 << bits):
            out = []
            for _ in range(nb - 1):
                out.append(0x80 | (v & 0x3F))
                v >>= 6
            return bytes([lead | v] + out[::-1])
    raise ValueError("number too large")


FIXED_COEFS = {0: [], 1: [1], 2: [2, -1], 3: [3, -3, 1], 4: [4, -6, 4, -1]}


def _residual(s: np.ndarray, coefs: Sequence[int], shift: int = 0) -> List[int]:
    p = len(coefs)
    out = []
    for i in range(p, len(s)):
        pred = sum(int(c) * int(s[i - 1 - j]) for j, c in enumerate(coefs))
        out.append(int(s[i]) - (pred >> shift))
    return out


def _write_residual(w: BitWriter, res: List[int], bs: int, order: int, porder: int, method: int, escape_parts=()):
    w.u(method, 2)
    w.u(porder, 4)
    pbits, esc = (4, 15) if method == 0 else (5, 31)
    parts = 1 << porder
    i = 0
    for pt in range(parts):
        cnt = (bs >> porder) - (order if pt == 0 else 0)
        chunk = res[i:i + cnt]
        i += cnt
        if pt in escape_parts:
            nb = max((max(abs(v) for v in chunk) if chunk else 0).bit_length() + 1, 0) if chunk else 0
            if chunk and all(v == 0 for v in chunk):
                nb = 0
            w.u(esc, pbits)
            w.u(nb, 5)
            for v in chunk:
                w.s(v, nb)
            continue
        zz = [(2 * v) if v >= 0 else (-2 * v - 1) for v in chunk]
        mean = (sum(zz) / len(zz)) if zz else 0
        k = 0
        while (1 << (k + 1)) <= mean + 1 and k < esc - 1:
            k += 1
        w.u(k, pbits)
        for z in zz:
            w.unary(z >> k)
            w.u(z & ((1 << k) - 1), k)


def encode_subframe(w: BitWriter, s: np.ndarray, bps: int, kind: str, order: int = 0, wasted: int = 0,
                    porder: int = 0, method: int = 0, escape_parts=(), lpc_prec: int = 12):
    """kind: 'constant' | 'verbatim' | 'fixed' | 'lpc'."""
    s = np.asarray(s, dtype=np.int64)
    bs = len(s)
    EMITTED.add((kind, order if kind in ("fixed", "lpc") else 0, bool(escape_parts) and kind in ("fixed", "lpc"),
                 method if kind in ("fixed", "lpc") else 0, wasted > 0))
    if wasted:
        assert np.all(s % (1 << wasted) == 0)
        s = s >> wasted
    eb = bps - wasted
    w.u(0, 1)
    if kind == "constant":
        assert np.all(s == s[0])
        w.u(0, 6)
    elif kind == "verbatim":
        w.u(1, 6)
    elif kind == "fixed":
        w.u(8 + order, 6)
    elif kind == "lpc":
        w.u(31 + order, 6)
    else:
        raise ValueError(kind)
    if wasted:
        w.u(1, 1)
        w.unary(wasted - 1)
    else:
        w.u(0, 1)
    if kind == "constant":
        w.s(int(s[0]), eb)
    elif kind == "verbatim":
        for v in s:
            w.s(int(v), eb)
    elif kind == "fixed":
        for v in s[:order]:
            w.s(int(v), eb)
        _write_residual(w, _residual(s, FIXED_COEFS[order]), bs, order, porder, method, escape_parts)
    else:  # lpc: least-squares predictor quantised to lpc_prec bits (any integer predictor is lossless)
        x = s.astype(np.float64)
        if bs > 2 * order:
            A = np.stack([x[order - 1 - j: bs - 1 - j] for j in range(order)], axis=1)
            a = np.linalg.lstsq(A, x[order:], rcond=None)[0]
        else:
            a = np.zeros(order)
        cmax = float(np.max(np.abs(a))) if order else 0.0
        shift = 0
        lim = (1 << (lpc_prec - 1)) - 1
        while shift < 15 and cmax * (1 << (shift + 1)) <= lim:
            shift += 1
        q = [int(max(-lim - 1, min(lim, round(c * (1 << shift))))) for c in a]
        for v in s[:order]:
            w.s(int(v), eb)
        w.u(lpc_prec - 1, 4)
        w.s(shift, 5)
        for c in q:
            w.s(c, lpc_prec)
        _write_residual(w, _residual(s, q, shift), bs, order, porder, method, escape_parts)


def block_size_code(bs: int):
    table = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12, 8192: 13,
             16384: 14, 32768: 15}
    if bs in table:
        return table[bs], b""
    if bs <= 256:
        return 6, bytes([bs - 1])
    return 7, struct.pack(">H", bs - 1)


RATE_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9, 48000: 10,
              96000: 11}
SIZE_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def encode(pcm: np.ndarray, rate: int, bps: int, block_sizes: Optional[Sequence[int]] = None, plan=None,
           variable: bool = False, rate_in_header: bool = True, size_in_header: bool = True, extra_meta: bool = True,
           total_known: bool = True) -> bytes:
    """pcm (C, T) integer samples.  plan(frame_index, channel) -> dict(kind, order, wasted, porder, method,
    escape_parts) and plan('stereo', frame_index) -> channel assignment 1 (independent) / 8 / 9 / 10."""
    pcm = np.asarray(pcm, dtype=np.int64)
    C, T = pcm.shape
    sizes = list(block_sizes or [4096])
    frames = []
    pos = fi = 0
    while pos < T:
        bs = min(sizes[fi % len(sizes)], T - pos)
        frames.append((pos, bs))
        pos += bs
        fi += 1
    max_bs = max(bs for _, bs in frames)
    min_bs = min(bs for _, bs in frames[:-1]) if len(frames) > 1 else max_bs
    out = bytearray(b"fLaC")
    si = BitWriter()
    si.u(max(16, min_bs if variable else max_bs), 16)
    si.u(max(16, max_bs), 16)
    si.u(0, 24)
    si.u(0, 24)
    si.u(rate, 20)
    si.u(C - 1, 3)
    si.u(bps - 1, 5)
    si.u(T if total_known else 0, 36)
    si.u(0, 128)
    blocks = [(0, si.bytes())]
    if extra_meta:
        blocks += [(4, struct.pack("<I", 4) + b"test" + struct.pack("<I", 0)), (1, bytes(37))]
    for i, (t, body) in enumerate(blocks):
        out += bytes([(0x80 if i == len(blocks) - 1 else 0) | t]) + len(body).to_bytes(3, "big") + body
    for fi, (p0, bs) in enumerate(frames):
        assign = plan("stereo", fi) if (plan and C == 2) else (C - 1)
        hdr = BitWriter()
        hdr.u(0x3FFE, 14)
        hdr.u(0, 1)
        hdr.u(1 if variable else 0, 1)
        bcode, bextra = block_size_code(bs)
        hdr.u(bcode, 4)
        rextra = b""
        if not rate_in_header:
            rcode = 0
        elif rate in RATE_CODES:
            rcode = RATE_CODES[rate]
        elif rate % 1000 == 0 and rate // 1000 < 256:
            rcode, rextra = 12, bytes([rate // 1000])
        elif rate < 65536:
            rcode, rextra = 13, struct.pack(">H", rate)
        else:
            rcode, rextra = 14, struct.pack(">H", rate // 10)
        hdr.u(rcode, 4)
        hdr.u(assign if C == 2 and assign in (8, 9, 10) else C - 1, 4)
        hdr.u(SIZE_CODES[bps] if size_in_header else 0, 3)
        hdr.u(0, 1)
        head = hdr.bytes() + utf8_number(p0 if variable else fi) + bextra + rextra
        head += bytes([crc8(head)])
        x = pcm[:, p0:p0 + bs]
        chans = [x[c] for c in range(C)]
        sbps = [bps] * C
        if C == 2 and assign == 8:
            chans, sbps = [x[0], x[0] - x[1]], [bps, bps + 1]
        elif C == 2 and assign == 9:
            chans, sbps = [x[0] - x[1], x[1]], [bps + 1, bps]
        elif C == 2 and assign == 10:
            chans, sbps = [(x[0] + x[1]) >> 1, x[0] - x[1]], [bps, bps + 1]
        w = BitWriter()
        for c in range(C):
            opts = dict(plan(fi, c)) if plan else dict(kind="fixed", order=2)
            if opts.get("kind") == "constant" and not np.all(chans[c] == chans[c][0]):
                opts = dict(kind="verbatim")
            if opts.get("kind") in ("fixed", "lpc") and opts.get("order", 0) > bs:
                opts = dict(kind="verbatim")
            porder = opts.get("porder", 0)
            order = opts.get("order", 0)
            while porder and ((bs % (1 << porder)) or (bs >> porder) < order):
                porder -= 1
            opts["porder"] = porder
            wasted = opts.get("wasted", 0)
            if wasted and not np.all(chans[c] % (1 << wasted) == 0):
                opts["wasted"] = 0
            encode_subframe(w, chans[c], sbps[c], **opts)
        w.align()
        frame = head + w.bytes()
        frame += struct.pack(">H", crc16(frame))
        out += frame
    return bytes(out)
