"""ctypes binding of libbigcodec_hip.so (the C ABI declared in include/bigcodec.h).

The HIP library IS the compute path: there is no eager-PyTorch or CPU fallback.  If the library is
missing or fails to load, every op raises immediately (BigCodecLibraryError).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading

import numpy as np

# BIGCODEC_DEBUG=1: the bounds-checked debug build (build_lib.build(debug=True), _debug/; include/bigcodec.h
# bc_debug_status) instead of the product library
# BIGCODEC_LIB_DIR: another build's directory (A/B timing of two builds on one box; tools/lab5/)
LIB_DIR = os.environ.get("BIGCODEC_LIB_DIR") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                             "_debug" if os.environ.get("BIGCODEC_DEBUG") == "1" else "")
_LIB_PATH = os.path.join(LIB_DIR, "libbigcodec_hip.so")
_lock = threading.Lock()
_lib = None

P = C.c_void_p
I = C.c_int
L = C.c_longlong

# name -> (restype, argtypes)
_SIGS = {
    "bc_abi_version": (I, []),
    "bc_build_digest": (C.c_char_p, []),
    "bc_conv1d_select_cfg": (I, [I, I, I, I, I, I]),
    "bc_conv1d_select_cfg_n": (I, [I, I, I, I, I, I, I, I]),
    "bc_conv1d_packed_floats": (L, [I, I, I, I]),
    "bc_conv1d_pack": (I, [P, P, I, I, I, I]),
    "bc_conv1d_fwd": (I, [P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, P]),
    "bc_resunit_select_cfg": (I, [I, I, I]),
    "bc_resunit_fwd": (I, [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, P]),
    "bc_resunit_fwd_snake_in": (I, [P] * 13 + [I] * 6 + [P]),
    "bc_convT1d_phase_taps": (I, [I, I]),
    "bc_convT1d_fwd": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, P]),
    "bc_convT1d_workspace_floats": (L, [I, I, I, I, I, I, I]),
    "bc_convT1d_fwd_ws": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, P, P]),
    "bc_snake_fwd": (I, [P, P, P, P, I, I, L, P]),
    "bc_aa_snake_fwd": (I, [P, P, P, P, P, P, I, I, I, P]),
    "bc_aa_snake_out_len": (L, [I, I, I, I]),
    "bc_aa_snake_fwd_ex": (I, [P, P, P, P, P, P, I, I, I, I, I, I, I, P]),
    "bc_lstm_hh_packed_floats": (L, [I, I]),
    "bc_lstm_pack_hh": (I, [P, P, I, I]),
    "bc_lstm_status": (I, [I]),
    "bc_mfma_probe": (I, [P, I, I, P]),
    "bc_lstm_workspace_floats": (L, [I, I, I]),
    "bc_reslstm_fwd": (I, [P, P, I, I, I, I, P, P, P, P, P, P, I, P]),
    "bc_reslstm_fwd_state": (I, [P, P, I, I, I, I, P, P, P, P, P, P, I, P, P, P, P, P]),
    "bc_reslstm_bidir_workspace_floats": (L, [I, I, I]),
    "bc_reslstm_bidir_fwd": (I, [P, P, I, I, I, I, P, P, P, P, P, P, I, P]),
    "bc_vq_prepare_codebook": (I, [P, P, P, I, I, P]),
    "bc_vq_fwd": (I, [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, P]),
    "bc_vq_argmin": (I, [P, P, P, P, L, I, I, P]),
    "bc_vq2emb": (I, [P, L, P, P, P, P, L, I, I, I, I, P]),
    "bc_vq2emb_ct": (I, [P, I, P, P, P, P, I, I, I, I, I, P]),
    "bc_fsq_fwd": (I, [P, P, P, P, P, P, P, P, I, I, I, I, P]),
    "bc_fsq_codes": (I, [P, I, P, P, P, P, I, I, I, I, P]),
    "bc_stream_window": (I, [P, L, L, P, P, P, P, P, I, I, I, I, P]),
    "bc_resample_sinc": (I, [P, P, P, I, L, L, L, I, I, I, I, P]),
    "bc_rvq_update": (I, [P, P, P, L, I, P]),
    "bc_btc_to_ctb": (I, [P, P, I, I, I, P]),
    "bc_ctb_to_btc_add": (I, [P, P, P, I, I, I, P]),
    "bc_synth_clips": (I, [P, I, L, L, P]),
    "bc_tanh_fwd": (I, [P, P, L, P]),
    "bc_flac_info": (I, [P, L, P, P, P, P]),
    "bc_flac_decode": (L, [P, L, P, I, L, I]),
    "bc_conv1d_kernel_name": (I, [I, I, I, I, C.c_char_p, I]),
    "bc_resunit_kernel_name": (I, [I, I, I, C.c_char_p, I]),
    "bc_debug_status": (I, [P]),
    "bc_debug_selftest": (I, [I, P]),
    "bc_launch_timer_enable": (I, [I]),
    "bc_launch_timer_read": (I, [I, C.c_char_p, P, P, P]),
}
EXPORTED = tuple(_SIGS)
# measurement-only entry points a library of an earlier ABI lacks (tools/lab* A/B runs load such builds through
# BIGCODEC_LIB_DIR); the product's own library exports them all (test_abi)
_OPTIONAL = ("bc_launch_timer_enable", "bc_launch_timer_read")
ABI_VERSION = 17  # include/bigcodec.h BC_ABI_VERSION

_ERR = {1: "bad argument", 2: "HIP launch error", 3: "unsupported shape"}


class BigCodecLibraryError(RuntimeError):
    pass


def lib_path() -> str:
    return _LIB_PATH


def load(path: str | None = None):
    """Load (once) and return the ctypes CDLL with argtypes set."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or _LIB_PATH
        if not os.path.exists(p):
            raise BigCodecLibraryError(
                f"{p} not found: build the HIP library first (python -c 'import __graft_entry__ as g; g.build()' "
                f"or python audiotokenization_amd/build_lib.py). There is no CPU/eager fallback.")
        try:
            lib = C.CDLL(p)
        except OSError as e:  # pragma: no cover - depends on the machine
            raise BigCodecLibraryError(f"failed to load {p}: {e}") from e
        for name, (res, args) in _SIGS.items():
            if name in _OPTIONAL and not hasattr(lib, name):
                continue  # an older build loaded for an A/B timing (BIGCODEC_LIB_DIR): timing hooks only
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise BigCodecLibraryError(f"{name} failed: {_ERR.get(rc, rc)} (code {rc})")


def call(name: str, *args) -> int:
    lib = load()
    rc = getattr(lib, name)(*args)
    check(rc, name)
    return rc


_tls = threading.local()  # per-thread status state: concurrent forwards on two threads never mix their words


def _pending():
    p = getattr(_tls, "pending", None)
    if p is None:
        p = _tls.pending = []
    return p


def defer_status(status, what: str) -> None:
    """Remember a device status word (nonzero = the launch failed, e.g. a persistent-kernel timeout,
    include/bigcodec.h) to be checked by check_status() before the caller's output is consumed."""
    _pending().append((status, what))


@contextlib.contextmanager
def status_scope():
    """Scope the deferred status words to one top-level forward: the body's launches defer into a fresh
    list, the body ends with check_status(); when the body raises instead, its unchecked words are dropped
    with it (that forward's output is never consumed), so a later forward cannot raise for a batch that
    already failed (a stale status after a per-batch error in the extraction loops).  Scopes
    nest: the enclosing forward's words are restored on exit.  The list is per thread."""
    outer = _pending()
    _tls.pending = []
    try:
        yield
    finally:
        _tls.pending = outer


def _raise_bad(items, vals) -> None:
    bad = [f"{what}: {v} workgroup(s) timed out" for (_, what), v in zip(items, vals) if v]
    if bad:
        raise BigCodecLibraryError("persistent LSTM launch failed, its output is wrong (" + "; ".join(bad) +
                                   "). The H/8 workgroups of the recurrence must be co-resident; another "
                                   "kernel holding CUs for seconds can starve them.")


def check_status() -> None:
    """Read every pending status word (ONE device -> host copy, which waits for the stream) and raise
    BigCodecLibraryError if any launch reported a failure.  Called at the end of each codec forward
    (encoder, decoder, streaming push, standalone ResLSTM).  Inside deferred_status() the words are handed
    to that scope's StatusTicket instead, and nothing waits for the device."""
    items = _pending()
    if not items:
        return
    _tls.pending = []
    coll = getattr(_tls, "deferred", None)
    if coll is not None:
        coll.extend(items)
        return
    import torch

    _raise_bad(items, torch.cat([t.reshape(-1) for t, _ in items]).cpu().tolist())


class StatusTicket:
    """The status words of the forwards run inside one deferred_status() scope, copied to pinned host memory
    behind the scope's work on the stream (no wait).  ready() polls, check() waits for the copy and raises
    BigCodecLibraryError like check_status() would have."""

    def __init__(self):
        self.items, self.host, self.event = [], None, None

    def _arm(self, items) -> None:
        import torch

        self.items = items
        if not items:
            return
        dev = items[0][0].device
        if dev.type != "cuda":  # host words (CPU test doubles): nothing to wait for
            self.host = torch.stack([t.reshape(-1)[0].to(torch.int32) for t, _ in items])
            return
        self.host = torch.empty(len(items), dtype=torch.int32, pin_memory=True)
        for i, (t, _) in enumerate(items):  # copies only: no compute kernel on the product path
            self.host[i:i + 1].copy_(t.reshape(-1)[:1].to(torch.int32), non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record(torch.cuda.current_stream(dev))

    def ready(self) -> bool:
        return self.event is None or self.event.query()

    def check(self) -> None:
        if self.event is not None:
            self.event.synchronize()
        if self.host is not None:
            _raise_bad(self.items, self.host.tolist())


@contextlib.contextmanager
def deferred_status():
    """Run forwards without their end-of-forward status read (a host wait for the whole forward): the words
    go to the yielded StatusTicket, armed when the body completes; the caller checks it before it uses the
    outputs (extract.ShardedExtractor checks batch i while batch i + 1 is queued on the device)."""
    items = []
    outer = getattr(_tls, "deferred", None)
    _tls.deferred = items
    ticket = StatusTicket()
    try:
        yield ticket
    finally:
        _tls.deferred = outer
    ticket._arm(items)


def conv_cfg(Cout: int, Cin: int, K: int, stride: int, dilation: int, mode: int) -> int:
    """bc_conv1d_select_cfg, checked: a negative answer (no tile for the shape) raises."""
    cfg = load().bc_conv1d_select_cfg(Cout, Cin, K, stride, dilation, mode)
    if cfg < 0:
        raise BigCodecLibraryError(f"bc_conv1d_select_cfg: no conv tile for Cout={Cout} Cin={Cin} K={K} "
                                   f"stride={stride} dilation={dilation} mode={mode} (returned {cfg})")
    return cfg


def checked_size(n: int, what: str) -> int:
    """A size query's answer (bc_*_packed_floats / bc_lstm_workspace_floats), checked: negative raises."""
    if n < 0:
        raise BigCodecLibraryError(f"{what} returned {n}: the shape or tile is not supported")
    return int(n)


def ptr(t) -> int | None:
    """Device (or host numpy) pointer of a tensor/array; None stays NULL."""
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


def stream_of(t) -> int | None:
    import torch

    if not t.is_cuda:
        raise BigCodecLibraryError("BigCodec HIP ops take device tensors (got a CPU tensor)")
    return torch.cuda.current_stream(t.device).cuda_stream


class KernelTimer:
    """Per-launch HIP-event timing of selected library calls (used by bench.py inside its timed
    region).  Events are recorded on the stream the kernel is launched on (torch's current stream,
    the one every op here passes to the library)."""

    def __init__(self):
        self.records = []  # (kernel symbol, flops, bytes, ev_start, ev_end)
        self.lib_records = []  # (kernel symbol, ms, flops, bytes): launches made inside the library's composite calls

    def drain_library(self):
        """Collect the library's own launch-timer records (bc_launch_timer_read: the ResLSTM transposes, projection
        and recurrence, the VQ), which the library brackets with HIP events on the launch stream."""
        lib = load()
        if not hasattr(lib, "bc_launch_timer_read"):
            return
        n = lib.bc_launch_timer_read(0, None, None, None, None)
        if n < 0:
            raise BigCodecLibraryError("bc_launch_timer_read failed")
        if n == 0:
            return
        names = C.create_string_buffer(64 * n)
        ms, fl, nb = (np.zeros(n, np.float32), np.zeros(n, np.float64), np.zeros(n, np.float64))
        got = lib.bc_launch_timer_read(n, names, ms.ctypes.data, fl.ctypes.data, nb.ctypes.data)
        if got < 0:
            raise BigCodecLibraryError("bc_launch_timer_read failed")
        raw = names.raw
        for i in range(min(n, got)):
            k = raw[64 * i:64 * (i + 1)].split(b"\0", 1)[0].decode()
            self.lib_records.append((k, float(ms[i]), float(fl[i]), float(nb[i])))

    def begin(self):
        import torch

        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def end(self, ev0, kernel: str, flops: float, nbytes: float):
        import torch

        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self.records.append((kernel, flops, nbytes, ev0, ev1))

    def summary(self):
        """{kernel: dict(launches, ms_total, flops_total, bytes_total)} (synchronises)."""
        import torch

        torch.cuda.synchronize()
        self.drain_library()
        out = {}
        rows = [(k, e0.elapsed_time(e1), fl, nb) for k, fl, nb, e0, e1 in self.records] + self.lib_records
        for k, ms, fl, nb in rows:
            d = out.setdefault(k, dict(launches=0, ms_total=0.0, flops_total=0.0, bytes_total=0.0))
            d["launches"] += 1
            d["ms_total"] += ms
            d["flops_total"] += fl
            d["bytes_total"] += nb
        return out


_timer: KernelTimer | None = None


def set_timer(t: KernelTimer | None) -> None:
    """Start (t) / stop (None) timing: the Python-dispatched launches into t, and the library's launch timer
    (bc_launch_timer_enable) for the launches inside its composite calls, drained into the timer that was active."""
    global _timer
    prev, _timer = _timer, t
    lib = load()
    if not hasattr(lib, "bc_launch_timer_enable"):
        return
    if prev is not None and prev is not t:
        lib.bc_launch_timer_enable(0)
        prev.drain_library()
    if t is not None and prev is not t:
        lib.bc_launch_timer_enable(1)


def active_timer() -> KernelTimer | None:
    return _timer


# conv tile configs (csrc/conv1d.hip kTiles x kBKC, cfg = tile*4 + bkc_index) -> template arguments
# (the packing-layout tables the ABI tests check; kernel NAMES come from the library, conv_kernel_name)
_TILES = [(4, 2, 4, 2), (4, 1, 4, 4), (3, 1, 4, 4), (2, 1, 4, 4), (1, 1, 4, 4)]
_BKC = [32, 16, 8, 4]
CONV_CFGS = {t * 4 + b: _TILES[t] + (_BKC[b],) for t in range(5) for b in range(4)}


# csrc/conv1d_x6.hip kX6Tiles (cfg = 100 + index) -> (MT, NT, WM, WN)
X6_CFGS = {100 + i: t for i, t in enumerate([(4, 4, 2, 4), (4, 2, 2, 4), (4, 2, 4, 2), (2, 2, 4, 2), (6, 2, 1, 8),
                                              (4, 2, 1, 8), (3, 2, 1, 8), (2, 2, 1, 8), (1, 2, 1, 8), (6, 1, 1, 8),
                                              (4, 1, 1, 8), (3, 1, 1, 8), (2, 1, 1, 8), (1, 1, 1, 8),
                                              (6, 2, 2, 4), (6, 1, 2, 4), (3, 1, 2, 4), (4, 1, 2, 4),
                                              (8, 2, 2, 4), (4, 4, 4, 2), (6, 4, 2, 4), (8, 4, 2, 4),
                                              (6, 2, 2, 8),  # 122: 16 waves (h3, bf16 and x6)
                                              (3, 2, 2, 4), (3, 4, 1, 8)])}  # 123, 124: one-launch ResidualUnit only


_name_cache = {}


def _kernel_name(fn: str, *args) -> str:
    key = (fn,) + args
    name = _name_cache.get(key)
    if name is None:
        buf = C.create_string_buffer(128)
        n = getattr(load(), fn)(*args, buf, 128)
        if n < 0:
            raise BigCodecLibraryError(f"{fn}{args}: invalid cfg")
        name = _name_cache[key] = buf.value.decode()
    return name


def conv_kernel_name(cfg: int, taps: int = 0, stride: int = 1, dilation: int = 1) -> str:
    """Kernel symbol a bc_conv1d_fwd launch with this cfg runs, as rocprofv3 prints it (without the
    namespace and arguments).  Decided by the launcher's own code (bc_conv1d_kernel_name), so the roofline
    attribution cannot drift from the tile table."""
    return _kernel_name("bc_conv1d_kernel_name", cfg, taps, stride, dilation)


def resunit_kernel_name(cfg: int, C: int = 0, dilation: int = 1) -> str:
    """Kernel symbol of a bc_resunit_fwd launch (bc_resunit_kernel_name)."""
    return _kernel_name("bc_resunit_kernel_name", cfg, C, dilation)


# Precision mode of the conv GEMMs: 0 = native fp32 MFMA, 1 = "x6", the default: both fp32 operands split EXACTLY
# into three bf16 terms (24-bit operands, the reference's fp32 width; vq/module.py:45-48, 65), six bf16 products per
# pair accumulated in fp32, at 2.65x the native fp32 MFMA ceiling,
# 2 = plain bf16 products (BASELINE config 5; NOT index-exact; the ResLSTM runs on h3: fp32-class, 22-bit operands),
# 3 = "h3": two fp16 planes per operand with power-of-two block scaling (22-bit operands: NARROWER than the
# reference's fp32), three products, at half the x6 MFMA count (opt-in: BIGCODEC_PRECISION=h3).
PRECISIONS = {"fp32": 0, "x6": 1, "bf16": 2, "h3": 3}
_mode = PRECISIONS[os.environ.get("BIGCODEC_PRECISION", "x6")]


def set_precision(name: str) -> None:
    """Select the conv GEMM arithmetic ('x6' default, 'fp32', 'h3', 'bf16'); prepared weights re-pack on next use."""
    global _mode
    if name not in PRECISIONS:
        raise ValueError(f"unknown precision {name!r}: expected one of {sorted(PRECISIONS)}")
    _mode = PRECISIONS[name]


def precision_mode() -> int:
    return _mode


def lstm_mode() -> int:
    """Mode the ResLSTM packs and runs with (bc_reslstm_fwd maps bf16 to h3: the recurrence stays fp32-class)."""
    return 3 if _mode == 2 else _mode


def precision_name() -> str:
    return {v: k for k, v in PRECISIONS.items()}[_mode]


def ptr_array(ptrs):
    arr = (C.c_void_p * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr


def debug_status():
    """(failed index checks, first failing source line) since the last call, from the bounds-checked debug
    build (BIGCODEC_DEBUG=1; synchronises the device), or None in the product build (no checks compiled)."""
    import torch

    torch.cuda.synchronize()
    out = (C.c_uint * 2)()
    rc = load().bc_debug_status(C.cast(out, C.c_void_p))
    if rc == 3:
        return None
    check(rc, "bc_debug_status")
    return int(out[0]), int(out[1])
