"""Composite blocks of the BigCodec stacks (vq/module.py:74-167) and the fused data flow.

Every conv in the reference is preceded by an Activation1d (Snake).  The HIP path computes each
Snake once, in the epilogue of the kernel that PRODUCES its input; a producer whose raw output is
still needed (as a ResidualUnit skip input) writes both raw and activated tensors.  The flow is
expressed with producer functions that take

    want_raw : does any consumer still need the raw output?
    next_act : the Activation1d that consumes the output (None: raw output only)

and return (raw or None, activated or None).  Anti-aliased activations (bc_aa_snake_fwd) cannot be
an epilogue; they run as their own kernel on the raw output.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch.nn import Parameter

from . import _lib as L
from . import ops
from .conv import WNConv1d, WNConvTranspose1d
from .modules import Activation1d, SnakeBeta, _DeviceCache, _as_input, _cpu, _pkey

__all__ = ["ResidualUnit", "EncoderBlock", "DecoderBlock", "LSTM", "ResLSTM"]

Flow = Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]


def _fusable(act: Optional[Activation1d]) -> bool:
    return act is not None and not act.antialias


def _conv_of(m):
    """The Conv1dWN behind a WNConv1d (CausalConv1d keeps it under `.conv`)."""
    return m.conv if hasattr(m, "conv") and not hasattr(m, "weight_v") else m


def produce_conv(conv, inp, residual=None, want_raw=True, next_act: Optional[Activation1d] = None,
                 epilogue: int = 0) -> Flow:
    """Run `conv` on an already-activated input and hand its output to `next_act`'s consumer."""
    if next_act is None:
        return conv.run(inp, residual, epilogue), None
    if _fusable(next_act):
        co = next_act.act.coeffs(inp.device)
        if want_raw:
            y, ya = conv.run(inp, residual, epilogue, out_snake=co, dual=True)
            return y, ya
        return None, conv.run(inp, residual, epilogue, out_snake=co)
    y = conv.run(inp, residual, epilogue)
    return y, next_act(y)


def produce_convT(conv, inp, want_raw=True, next_act: Optional[Activation1d] = None) -> Flow:
    if next_act is None:
        return conv.run(inp), None
    if _fusable(next_act):
        co = next_act.act.coeffs(inp.device)
        if want_raw:
            return conv.run(inp, out_snake=co, dual=True)
        return None, conv.run(inp, out_snake=co)
    y = conv.run(inp)
    return y, next_act(y)


class ResidualUnit(nn.Module):
    """vq/module.py:74-89: x + conv1(act2(conv7_d(act1(x)))).  Two launches: conv7 (epilogue =
    act2), conv1 (epilogue = skip add [+ the next block's Snake])."""

    def __init__(self, dim: int = 16, dilation: int = 1, causal: bool = False, antialias: bool = False):
        super().__init__()
        pad = 0 if causal else ((7 - 1) * dilation) // 2
        self.block = nn.Sequential(
            Activation1d(activation=SnakeBeta(dim, alpha_logscale=True), antialias=antialias),
            WNConv1d(dim, dim, kernel_size=7, dilation=dilation, padding=pad, causal=causal),
            Activation1d(activation=SnakeBeta(dim, alpha_logscale=True), antialias=antialias),
            WNConv1d(dim, dim, kernel_size=1),
        )

    @property
    def first_act(self) -> Activation1d:
        return self.block[0]

    def _fused_cfg(self):
        """cfg of the one-launch unit (bc_resunit_fwd), or -1 (x6 / bf16 / h3 mode, no anti-aliasing, C fits)."""
        mode = L.precision_mode()
        if mode not in (1, 2, 3) or self.block[2].antialias:
            return -1
        conv7 = _conv_of(self.block[1])
        return L.load().bc_resunit_select_cfg(conv7.in_channels, conv7.dilation, mode)

    def snake_on_load(self) -> bool:
        """True when the one-launch kernel applies the first Snake while staging its input
        (bc_resunit_fwd_snake_in): the producer then writes the raw tensor only (x_act=None).
        BIGCODEC_RU_SNAKE_IN=0 restores producer-side activation (dual raw + activated outputs)."""
        if not _fusable(self.first_act) or os.environ.get("BIGCODEC_RU_SNAKE_IN", "1") == "0":
            return False
        return self._fused_cfg() >= 0

    def flow(self, x_raw, x_act, want_raw=True, next_act=None) -> Flow:
        """x_act = self.first_act(x_raw) computed by the producer, or None (snake_on_load)."""
        if next_act is None or _fusable(next_act):
            cfg = self._fused_cfg()
            if cfg >= 0:
                return self._flow_fused(cfg, x_raw, x_act, want_raw, next_act)
        if x_act is None:
            x_act = self.first_act(x_raw)
        _, h = produce_conv(self.block[1], x_act, None, want_raw=False, next_act=self.block[2])
        return produce_conv(self.block[3], h, residual=x_raw, want_raw=want_raw, next_act=next_act)

    def _flow_fused(self, cfg, x_raw, x_act, want_raw, next_act) -> Flow:
        conv7, conv1 = _conv_of(self.block[1]), _conv_of(self.block[3])
        lazy = x_act is None and _fusable(self.first_act)
        if x_act is None and not lazy:
            x_act = self.first_act(x_raw)
        dev = x_raw.device
        w7, b7 = conv7.packed_as(cfg, dev)
        w1, b1 = conv1.packed_as(cfg, dev)
        s2a, s2b = self.block[2].act.coeffs(dev)
        B, C, T = x_raw.shape
        if not lazy and x_raw.shape != x_act.shape:
            raise ValueError("ResidualUnit: raw and activated inputs differ in shape")
        sa, sb = next_act.act.coeffs(dev) if next_act is not None else (None, None)
        dual = next_act is not None and want_raw
        tm = L.active_timer()
        ev = tm.begin() if tm is not None else None
        s1a, s1b = self.first_act.act.coeffs(dev) if lazy else (None, None)
        out = ops.load().resunit(x_raw, None if lazy else x_act, s1a, s1b, w7, b7, s2a, s2b, w1, b1, sa, sb,
                                 conv7.dilation, conv7.pad_left(), cfg, dual)
        y, y2 = out[0], (out[1] if dual else None)
        if tm is not None:
            flops = 2.0 * B * C * C * T * 8  # k=7 and k=1
            nbytes = 4.0 * x_raw.numel() * ((2 if lazy else 3) + dual)
            tm.end(ev, L.resunit_kernel_name(cfg, C, conv7.dilation), flops, nbytes)
        if next_act is None:
            return y, None
        if dual:
            return y, y2
        return None, y

    def forward(self, x):
        x = _as_input(x)
        return self.flow(x, None if self.snake_on_load() else self.first_act(x))[0]


def input_act(stage) -> Optional[Activation1d]:
    """The activation a producer must apply for `stage` (a ResidualUnit / Encoder- / DecoderBlock);
    None when the stage's first ResidualUnit activates on load (raw output only)."""
    first = stage if isinstance(stage, ResidualUnit) else stage.block[0]
    if isinstance(first, ResidualUnit) and first.snake_on_load():
        return None
    return stage.first_act


class EncoderBlock(nn.Module):
    """vq/module.py:91-113: ResidualUnits -> Activation1d -> strided conv (k=2s) C/2 -> C."""

    def __init__(self, dim: int = 16, stride: int = 1, dilations=(1, 3, 9), causal: bool = False,
                 antialias: bool = False):
        super().__init__()
        runits = [ResidualUnit(dim // 2, dilation=d, causal=causal, antialias=antialias) for d in dilations]
        pad = 0 if causal else (stride // 2 + stride % 2 if stride != 1 else 0)
        self.block = nn.Sequential(
            *runits,
            Activation1d(activation=SnakeBeta(dim // 2, alpha_logscale=True), antialias=antialias),
            WNConv1d(dim // 2, dim, kernel_size=2 * stride if stride != 1 else 1, stride=stride, padding=pad,
                     causal=causal),
        )

    @property
    def first_act(self) -> Activation1d:
        return self.block[0].first_act

    def flow(self, x_raw, x_act, want_raw=True, next_act=None) -> Flow:
        n = len(self.block)
        rus = [self.block[i] for i in range(n - 2)]
        for i, ru in enumerate(rus):
            last = i == len(rus) - 1
            nxt = self.block[n - 2] if last else input_act(rus[i + 1])
            x_raw, x_act = ru.flow(x_raw, x_act, want_raw=not last, next_act=nxt)
        return produce_conv(self.block[n - 1], x_act, None, want_raw=want_raw, next_act=next_act)

    def forward(self, x):
        x = _as_input(x)
        return self.flow(x, None if input_act(self) is None else self.first_act(x))[0]


class DecoderBlock(nn.Module):
    """vq/module.py:115-141: Activation1d -> transposed conv (k=2s) -> ResidualUnits."""

    def __init__(self, input_dim: int = 16, output_dim: int = 8, stride: int = 1, dilations=(1, 3, 9),
                 causal: bool = False, antialias: bool = False):
        super().__init__()
        if causal:
            tconv_kwargs = {}
        else:
            tconv_kwargs = {"padding": stride // 2 + stride % 2 if stride != 1 else 0,
                            "output_padding": stride % 2 if stride != 1 else 0}
        self.block = nn.Sequential(
            Activation1d(activation=SnakeBeta(input_dim, alpha_logscale=True), antialias=antialias),
            WNConvTranspose1d(input_dim, output_dim, kernel_size=2 * stride if stride != 1 else 1, stride=stride,
                              causal=causal, **tconv_kwargs),
        )
        self.block.extend([ResidualUnit(output_dim, dilation=d, causal=causal, antialias=antialias)
                           for d in dilations])

    @property
    def first_act(self) -> Activation1d:
        return self.block[0]

    def flow(self, x_raw, x_act, want_raw=True, next_act=None) -> Flow:
        rus = [self.block[i] for i in range(2, len(self.block))]
        y_raw, y_act = produce_convT(self.block[1], x_act, want_raw=True,
                                     next_act=input_act(rus[0]) if rus else next_act)
        for i, ru in enumerate(rus):
            last = i == len(rus) - 1
            y_raw, y_act = ru.flow(y_raw, y_act, want_raw=(want_raw if last else True),
                                   next_act=next_act if last else input_act(rus[i + 1]))
        return y_raw, y_act

    def forward(self, x):
        x = _as_input(x)
        return self.flow(x, self.first_act(x))[0]


class LSTM(nn.Module):
    """Parameter container with torch.nn.LSTM's names (weight_ih_l{k}, weight_hh_l{k}, bias_ih_l{k},
    bias_hh_l{k}; batch_first) so reference checkpoints load; the recurrence runs in
    bc_reslstm_fwd."""

    def __init__(self, input_size, hidden_size, num_layers=1, bias=True, batch_first=True, dropout=0.0,
                 bidirectional=False):
        super().__init__()
        if not bias or not batch_first or dropout:
            raise NotImplementedError("only bias=True, batch_first=True, dropout=0")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.batch_first, self.bidirectional = batch_first, bidirectional
        ref = nn.LSTM(input_size, hidden_size, num_layers, batch_first=True,
                      bidirectional=bidirectional)  # torch's default init and parameter names
        for name, p in ref.named_parameters():
            setattr(self, name, Parameter(p.detach().clone()))
        self._cache = _DeviceCache()

    def _suffixes(self):
        return ("", "_reverse") if self.bidirectional else ("",)

    def _plist(self):
        out = []
        for l in range(self.num_layers):
            for sfx in self._suffixes():
                out += [getattr(self, f"weight_ih_l{l}{sfx}"), getattr(self, f"weight_hh_l{l}{sfx}"),
                        getattr(self, f"bias_ih_l{l}{sfx}"), getattr(self, f"bias_hh_l{l}{sfx}")]
        return out

    def prepared(self, device):
        """Packed per-layer weights; bidirectional: [forward, backward] per layer (bc_reslstm_bidir_fwd)."""
        def build():
            lib = L.load()
            H = self.hidden_size
            # unidirectional: the residual needs input == hidden; bidirectional: every layer reads the
            # 2H-channel concatenation, so the module input must be 2H as well
            Cin = 2 * H if self.bidirectional else H
            if self.input_size != Cin:
                raise NotImplementedError("ResLSTM requires input_size == hidden_size (x2 when bidirectional)")
            mode = L.lstm_mode()
            cfg = L.conv_cfg(4 * H, Cin, 1, 1, 1, mode)
            wih, whh, bias = [], [], []
            for l in range(self.num_layers):
                for sfx in self._suffixes():
                    w = _cpu(getattr(self, f"weight_ih_l{l}{sfx}")).contiguous()
                    packed = np.empty(L.checked_size(lib.bc_conv1d_packed_floats(4 * H, Cin, 1, cfg),
                                                     "bc_conv1d_packed_floats"), dtype=np.float32)
                    L.call("bc_conv1d_pack", w.numpy().ctypes.data, packed.ctypes.data, 4 * H, Cin, 1, cfg)
                    wih.append(torch.from_numpy(packed).to(device))
                    w = _cpu(getattr(self, f"weight_hh_l{l}{sfx}")).contiguous()
                    packed = np.empty(L.checked_size(lib.bc_lstm_hh_packed_floats(H, mode), "bc_lstm_hh_packed_floats"),
                                      dtype=np.float32)
                    L.call("bc_lstm_pack_hh", w.numpy().ctypes.data, packed.ctypes.data, H, mode)
                    whh.append(torch.from_numpy(packed).to(device))
                    b = _cpu(getattr(self, f"bias_ih_l{l}{sfx}")) + _cpu(getattr(self, f"bias_hh_l{l}{sfx}"))
                    bias.append(b.contiguous().to(device))
            arrs = (L.ptr_array([t.data_ptr() for t in wih]), L.ptr_array([t.data_ptr() for t in bias]),
                    L.ptr_array([t.data_ptr() for t in whh]))
            return (wih, whh, bias), arrs
        return self._cache.get(_pkey(*self._plist()) + (str(device), L.lstm_mode()), build)


class ResLSTM(nn.Module):
    """vq/module.py:143-167: y = LSTM(x^T)^T + x for x (B, F, T)."""

    def __init__(self, dimension: int, num_layers: int = 2, bidirectional: bool = False, skip: bool = True):
        super().__init__()
        if not skip:
            raise NotImplementedError("ResLSTM(skip=False) is not used by the reference models")
        self.skip = skip
        self.lstm = LSTM(dimension, dimension if not bidirectional else dimension // 2, num_layers,
                         batch_first=True, bidirectional=bidirectional)

    def run(self, x, out_snake=None, state=None, return_state: bool = False):
        """y = LSTM(x^T)^T + x (then the next Snake when out_snake = (alpha_exp, inv_beta)).  Streaming:
        state = (h0, c0) [num_layers][H][B] device tensors or None (zeros); with return_state the call
        returns (y, (h_n, c_n)) in the same layout (nn.LSTM's final state, unit-major)."""
        x = _as_input(x)
        B, H, T = x.shape
        (wih, whh, bias), _ = self.lstm.prepared(x.device)
        sa, sb = out_snake if out_snake is not None else (None, None)
        if self.lstm.bidirectional:
            if state is not None or return_state:
                raise NotImplementedError("carried state (streaming) needs a unidirectional ResLSTM")
            out = ops.load().reslstm_bidir(x, wih, bias, whh, sa, sb, L.precision_mode())
            L.defer_status(out[1], f"ResLSTM(D={H}, layers={self.lstm.num_layers}, bidirectional, T={T})")
            return out[0]
        h0, c0 = state if state is not None else (None, None)
        out = ops.load().reslstm(x, wih, bias, whh, sa, sb, L.precision_mode(), h0, c0, return_state)
        # include/bigcodec.h: out[1] = the call's count of persistent workgroups that timed out; the
        # codec's forward checks it (L.check_status) before its output can be consumed
        L.defer_status(out[1], f"ResLSTM(H={H}, layers={self.lstm.num_layers}, T={T})")
        if return_state:
            return out[0], (out[2], out[3])
        return out[0]

    def flow(self, x_raw, want_raw=True, next_act=None) -> Flow:
        if next_act is None:
            return self.run(x_raw), None
        if _fusable(next_act) and not want_raw:
            return None, self.run(x_raw, out_snake=next_act.act.coeffs(x_raw.device))
        y = self.run(x_raw)
        return y, next_act(y)

    def forward(self, x):
        with L.status_scope():
            y = self.run(x)
            L.check_status()
        return y
