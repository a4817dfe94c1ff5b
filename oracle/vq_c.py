"""ctypes wrapper of the C VQ oracle — TEST INFRASTRUCTURE ONLY."""
import ctypes as C

import numpy as np

from . import build as _build

_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(_build.build())
        _lib.vq_oracle_prepare.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _lib.vq_oracle_argmin.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_longlong, C.c_int,
                                          C.c_void_p, C.c_void_p, C.c_void_p]
    return _lib


def prepare(codebook: np.ndarray):
    cb = np.ascontiguousarray(codebook, dtype=np.float32)
    cbn = np.empty_like(cb)
    csq = np.empty(cb.shape[0], np.float32)
    lib().vq_oracle_prepare(cb.ctypes.data, cbn.ctypes.data, csq.ctypes.data, cb.shape[0])
    return cbn, csq


def argmin(z_e: np.ndarray, codebook: np.ndarray, return_dists: bool = False):
    ze = np.ascontiguousarray(z_e, dtype=np.float32).reshape(-1, 8)
    cbn, csq = prepare(codebook)
    n = ze.shape[0]
    idx = np.empty(n, np.int64)
    best = np.empty(n, np.float32)
    second = np.empty(n, np.float32)
    lib().vq_oracle_argmin(ze.ctypes.data, cbn.ctypes.data, csq.ctypes.data, n, cbn.shape[0], idx.ctypes.data,
                           best.ctypes.data, second.ctypes.data)
    if return_dists:
        return idx, best, second
    return idx
