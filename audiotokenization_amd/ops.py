"""torch.ops.bigcodec.* — the PyTorch-ROCm custom operators of the BigCodec path (BASELINE.json north_star:
"surfaced as PyTorch-ROCm custom ops"; SURVEY.md §8(b) TORCH_LIBRARY(bigcodec)).

libbigcodec_ops.so (csrc/torch_ops.cpp, built by build_lib.build_ops) registers the schemas and the HIP
implementations over the C ABI of libbigcodec_hip.so.  This module loads it and registers the fake
(shape-only) kernels used by FakeTensor tracing, torch.compile and torch.library.opcheck.  The codec
modules (conv.py, blocks.py, modules.py, codec.py, ingest.py, extract.py) call these ops; there is no
eager-PyTorch or CPU fallback: a missing library raises BigCodecLibraryError.

    import audiotokenization_amd.ops as ops
    y = ops.load().snake(x, alpha_exp, inv_beta)           # == torch.ops.bigcodec.snake(...)
"""
from __future__ import annotations

import os
import threading

import torch

from . import _lib as L

OPS_PATH = os.path.join(L.LIB_DIR, "libbigcodec_ops.so")  # next to the libbigcodec_hip.so it links ($ORIGIN)
_lock = threading.Lock()
_ns = None

# every op the extension defines (tests check the registry against this list)
OPS = ("conv1d", "conv_transpose1d", "resunit", "snake", "aa_snake", "aa_snake_ex", "tanh", "reslstm", "reslstm_bidir", "vq_prepare_codebook", "vq",
       "vq_argmin", "vq2emb", "vq2emb_add_", "rvq_update_", "vq2emb_ct", "fsq", "fsq_codes", "stream_window", "resample_sinc", "synth_clips_")


def load():
    """Load libbigcodec_ops.so once (after the C-ABI library) and return the torch.ops.bigcodec namespace."""
    global _ns
    if _ns is not None:
        return _ns
    with _lock:
        if _ns is None:
            L.load()
            if not os.path.exists(OPS_PATH):
                raise L.BigCodecLibraryError(
                    f"{OPS_PATH} not found: build it (python -c 'import __graft_entry__ as g; g.build()'). "
                    f"There is no CPU/eager fallback.")
            torch.ops.load_library(OPS_PATH)
            _register_fakes()
            _ns = torch.ops.bigcodec
    return _ns


def _new(like, shape, dtype=torch.float32):
    return like.new_empty(shape, dtype=dtype)


def _register_fakes():
    reg = torch.library.register_fake

    @reg("bigcodec::conv1d")
    def _conv1d(x, w_packed, bias, residual, sa, sb, cout, tout, kernel_size, stride, dilation, pad_left, epilogue,
                cfg, dual):
        y = _new(x, (x.shape[0], cout, tout))
        return [y, _new(x, y.shape)] if dual else [y]

    @reg("bigcodec::conv_transpose1d")
    def _convt(x, w_phases, bias, sa, sb, cout, tout, kernel_size, stride, padding, cfg, dual):
        y = _new(x, (x.shape[0], cout, tout))
        return [y, _new(x, y.shape)] if dual else [y]

    @reg("bigcodec::resunit")
    def _resunit(x_raw, x_act, ia, ib, w7, b7, ma, mb, w1, b1, oa, ob, dilation, pad_left, cfg, dual):
        return [_new(x_raw, x_raw.shape), _new(x_raw, x_raw.shape)] if dual else [_new(x_raw, x_raw.shape)]

    @reg("bigcodec::snake")
    def _snake(x, a, ib):
        return _new(x, x.shape)

    @reg("bigcodec::aa_snake")
    def _aa(x, a, ib, fu, fd):
        return _new(x, x.shape)

    @reg("bigcodec::aa_snake_ex")
    def _aa_ex(x, a, ib, fu, fd, up_ratio, down_ratio):
        kd = fd.numel()
        L = x.shape[2] * up_ratio
        n = L + (kd // 2 - (1 if kd % 2 == 0 else 0)) + kd // 2 - kd
        return _new(x, (x.shape[0], x.shape[1], n // down_ratio + 1 if n >= 0 else 0))

    @reg("bigcodec::tanh")
    def _tanh(x):
        return _new(x, x.shape)

    @reg("bigcodec::reslstm")
    def _reslstm(x, w_ih, bias, w_hh, sa, sb, mode, h0, c0, return_state):
        out = [_new(x, x.shape), _new(x, (1,), torch.int32)]
        if return_state or h0 is not None:
            B, H, _ = x.shape
            out += [_new(x, (len(w_ih), H, B)), _new(x, (len(w_ih), H, B))]
        return out

    @reg("bigcodec::reslstm_bidir")
    def _reslstm_bidir(x, w_ih, bias, w_hh, sa, sb, mode):
        return [_new(x, x.shape), _new(x, (1,), torch.int32)]

    @reg("bigcodec::vq_prepare_codebook")
    def _prep(cb):
        return [_new(cb, cb.shape), _new(cb, (cb.shape[0],))]

    @reg("bigcodec::vq")
    def _vq(z, w_in, b_in, cb, cbn, cbsq, w_out, b_out, want_ze, want_post):
        B, D, T = z.shape
        out = [_new(z, (B, T), torch.int64)]
        if want_ze:
            out.append(_new(z, (B, cb.shape[1], T)))
        if want_post:
            out.append(_new(z, z.shape))
        return out

    @reg("bigcodec::vq_argmin")
    def _argmin(ze, cbn, cbsq):
        return _new(ze, (ze.shape[0],), torch.int64)

    @reg("bigcodec::vq2emb")
    def _vq2emb(idx, column, cb, w_out, b_out):
        D = w_out.shape[0] if w_out is not None else cb.shape[1]
        return _new(idx, tuple(idx.shape[:-1]) + (D,))

    @reg("bigcodec::vq2emb_add_")
    def _vq2emb_add(out, idx, column, cb, w_out, b_out):
        return None

    @reg("bigcodec::rvq_update_")
    def _rvq(residual, out, q, first):
        return None

    @reg("bigcodec::vq2emb_ct")
    def _vq2emb_ct(idx, cbs, w_out, b_out):
        B, T, _ = idx.shape
        return _new(idx, (B, w_out.shape[1], T))

    @reg("bigcodec::fsq")
    def _fsq(z, w_in, b_in, w_out, b_out, consts):
        B, D, T = z.shape
        return [_new(z, z.shape), _new(z, (B, T), torch.int32)]

    @reg("bigcodec::fsq_codes")
    def _fsq_codes(idx, w_out, b_out, levels):
        B, T = idx.shape
        return _new(idx, (B, b_out.shape[0], T), torch.float32)

    @reg("bigcodec::stream_window")
    def _stream_window(x, ctx, a, ib, P):
        B, C, n = x.shape
        return [_new(x, (B, C, P + n)), _new(x, (B, C, P))]

    @reg("bigcodec::resample_sinc")
    def _resample(x, kern, lout, pitch, orig, new_freq, taps, width):
        return _new(x, tuple(x.shape[:-1]) + (pitch,))

    @reg("bigcodec::synth_clips_")
    def _synth(x, clip0):
        return None
