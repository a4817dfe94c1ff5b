"""Weight-normed Conv1d / ConvTranspose1d modules (vq/module.py:11-72) on bc_conv1d_fwd /
bc_convT1d_fwd.  Parameter names and constructor signatures are those of
torch.nn.utils.weight_norm(nn.Conv1d / nn.ConvTranspose1d) and of the reference's CausalConv1d /
CausalConvTranspose1d wrappers, so reference state_dicts load strictly.

`run()` exposes the fused epilogue: residual add, tanh, or the Snake of the next Activation1d
(alone, or beside the raw value: dual output)."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn as nn
from torch.nn import Parameter

from . import _lib as L
from . import ops
from .modules import _DeviceCache, _as_input, _cpu, _pkey

__all__ = ["Conv1dWN", "CausalConv1d", "WNConv1d", "ConvTranspose1dWN", "CausalConvTranspose1d",
           "WNConvTranspose1d"]


def _wn_init(module: nn.Module, ref_weight: torch.Tensor, ref_bias: Optional[torch.Tensor]):
    """weight_norm's initial state: weight_v = weight, weight_g = ||weight|| over dims != 0."""
    if ref_bias is not None:
        module.bias = Parameter(ref_bias.detach().clone())
    else:
        module.register_parameter("bias", None)
    v = ref_weight.detach().clone()
    g = torch.linalg.vector_norm(v.reshape(v.shape[0], -1), dim=1).reshape((-1,) + (1,) * (v.dim() - 1))
    module.weight_g = Parameter(g)
    module.weight_v = Parameter(v)


class _WNParams:
    """Shared weight-norm parameter helpers (fold once on the host with torch._weight_norm — the
    function the reference's forward pre-hook evaluates — so folded weights are bit-identical)."""

    def folded_weight(self) -> torch.Tensor:
        if "weight" in self._parameters:
            return _cpu(self._parameters["weight"])
        return torch._weight_norm(_cpu(self.weight_v), _cpu(self.weight_g), 0)

    def remove_weight_norm(self):
        w = self.folded_weight()
        del self._parameters["weight_g"]
        del self._parameters["weight_v"]
        self.weight = Parameter(w.to(self.bias.device if self.bias is not None else "cpu"))

    def _params(self):
        if "weight" in self._parameters:
            return (self._parameters["weight"], self.bias)
        return (self.weight_g, self.weight_v, self.bias)


def _epilogue_args(out_snake, dual):
    if out_snake is None:
        if dual:
            raise ValueError("dual output needs an out_snake")
        return None, None
    return out_snake


class Conv1dWN(_WNParams, nn.Module):
    """weight_norm(nn.Conv1d(...)): parameters bias, weight_g (Cout,1,1), weight_v (Cout,Cin,K)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode="zeros", device=None, dtype=None):
        super().__init__()
        if groups != 1 or padding_mode != "zeros":
            raise NotImplementedError("only groups=1, padding_mode='zeros' (all the reference uses)")
        if isinstance(padding, str):
            raise NotImplementedError("string padding is not used by the reference")
        one = lambda v: int(v[0] if isinstance(v, (tuple, list)) else v)  # noqa: E731
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride = one(kernel_size), one(stride)
        self.padding, self.dilation = one(padding), one(dilation)
        self.causal_pad: Optional[int] = None  # set by CausalConv1d
        ref = nn.Conv1d(in_channels, out_channels, self.kernel_size, bias=bias)
        _wn_init(self, ref.weight, ref.bias)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()  # the reference's init_weights zeroes conv biases
        self._cache = _DeviceCache()

    def prepared(self, device):
        def build():
            w = self.folded_weight().contiguous()
            Cout, Cin, K = w.shape
            lib = L.load()
            cfg = L.conv_cfg(Cout, Cin, K, self.stride, self.dilation, L.precision_mode())
            packed = np.empty(L.checked_size(lib.bc_conv1d_packed_floats(Cout, Cin, K, cfg),
                                             f"bc_conv1d_packed_floats({Cout}, {Cin}, {K}, cfg {cfg})"), dtype=np.float32)
            L.call("bc_conv1d_pack", w.numpy().ctypes.data, packed.ctypes.data, Cout, Cin, K, cfg)
            bias = _cpu(self.bias).contiguous().to(device) if self.bias is not None else None
            return torch.from_numpy(packed).to(device), bias, cfg
        return self._cache.get(_pkey(*self._params()) + (str(device), L.precision_mode()), build)

    def packed_as(self, cfg: int, device):
        """(packed weight, bias) for an explicit cfg (the fused ResidualUnit's tile)."""
        def build():
            w = self.folded_weight().contiguous()
            Cout, Cin, K = w.shape
            lib = L.load()
            packed = np.empty(L.checked_size(lib.bc_conv1d_packed_floats(Cout, Cin, K, cfg),
                                             f"bc_conv1d_packed_floats({Cout}, {Cin}, {K}, cfg {cfg})"), dtype=np.float32)
            L.call("bc_conv1d_pack", w.numpy().ctypes.data, packed.ctypes.data, Cout, Cin, K, cfg)
            bias = _cpu(self.bias).contiguous().to(device) if self.bias is not None else None
            return torch.from_numpy(packed).to(device), bias
        if not hasattr(self, "_cache_as"):
            self._cache_as = {}
        return self._cache_as.setdefault(cfg, _DeviceCache()).get(_pkey(*self._params()) + (str(device), cfg), build)

    def pad_left(self) -> int:
        return self.causal_pad if self.causal_pad is not None else self.padding

    def out_len(self, T: int, pad_left: Optional[int] = None) -> int:
        if pad_left is not None:  # explicit left pad, none on the right (streaming with carried context)
            return (T + pad_left - self.dilation * (self.kernel_size - 1) - 1) // self.stride + 1
        pr = 0 if self.causal_pad is not None else self.padding
        return (T + self.pad_left() + pr - self.dilation * (self.kernel_size - 1) - 1) // self.stride + 1

    def run(self, x, residual=None, epilogue: int = 0, out_snake=None, dual: bool = False,
            pad_left: Optional[int] = None):
        """y = conv(x) + bias [+ residual]; then tanh (epilogue=1) or the next Snake (out_snake =
        (alpha_exp, inv_beta)).  Returns y, or (raw, snake(raw)) when dual.  pad_left overrides the
        module's padding (left only; streaming.py passes 0 with the carried context prepended)."""
        x = _as_input(x)
        B, Cin, T = x.shape
        if Cin != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {Cin}")
        wp, bias, cfg = self.prepared(x.device)
        pl = self.pad_left() if pad_left is None else pad_left
        Tout = self.out_len(T, pad_left)
        if Tout <= 0:
            raise ValueError(f"input length {T} too short for this convolution")
        if residual is not None:
            residual = _as_input(residual)
            if tuple(residual.shape) != (B, self.out_channels, Tout):
                raise ValueError(f"residual shape {tuple(residual.shape)} != output {(B, self.out_channels, Tout)}")
        sa, sb = _epilogue_args(out_snake, dual)
        if Tout <= 128:  # a narrow launch may take a narrower tile
            cfg_n = L.load().bc_conv1d_select_cfg_n(self.out_channels, Cin, self.kernel_size, self.stride,
                                                    self.dilation, L.precision_mode(), B, Tout)
            if cfg_n >= 0 and cfg_n != cfg:
                wp, bias = self.packed_as(cfg_n, x.device)
                cfg = cfg_n
        tm = L.active_timer()
        ev = tm.begin() if tm is not None else None
        out = ops.load().conv1d(x, wp, bias, residual, sa, sb, self.out_channels, Tout, self.kernel_size, self.stride,
                                self.dilation, pl, epilogue, cfg, dual)
        y, y2 = out[0], (out[1] if dual else None)
        if tm is not None:
            flops = 2.0 * B * self.out_channels * Cin * self.kernel_size * Tout
            nbytes = 4.0 * (x.numel() + y.numel() * (1 + (residual is not None) + dual))
            tm.end(ev, L.conv_kernel_name(cfg, self.kernel_size, self.stride, self.dilation), flops, nbytes)
        return (y, y2) if dual else y

    def forward(self, x):
        return self.run(x)


class CausalConv1d(nn.Module):
    """vq/module.py:11-48: left zero-pad (k - s) * d, then conv; parameters under `.conv`."""

    def __init__(self, in_channels, out_channels, kernel_size, padding=0, stride=1, dilation=1, groups=1,
                 bias=True, padding_mode="zeros", device=None, dtype=None):
        super().__init__()
        self.conv = Conv1dWN(in_channels, out_channels, kernel_size, stride=stride, padding=0,
                             dilation=dilation, groups=groups, bias=bias)
        self.padding_mode = "constant" if padding_mode == "zeros" else padding_mode
        self.padding = (kernel_size - stride) * dilation
        self.conv.causal_pad = self.padding

    def run(self, x, residual=None, epilogue: int = 0, out_snake=None, dual: bool = False):
        return self.conv.run(x, residual, epilogue, out_snake, dual)

    def forward(self, x):
        return self.conv.run(x)

    @property
    def in_channels(self):
        return self.conv.in_channels

    @property
    def out_channels(self):
        return self.conv.out_channels


def WNConv1d(*args, causal=False, **kwargs):
    """vq/module.py:59-65."""
    if causal:
        return CausalConv1d(*args, **kwargs)
    return Conv1dWN(*args, **kwargs)


class ConvTranspose1dWN(_WNParams, nn.Module):
    """weight_norm(nn.ConvTranspose1d(...)): weight_v (Cin, Cout, K), weight_g (Cin, 1, 1) — the norm
    runs over dim 0 = INPUT channels — and bias (Cout)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0,
                 groups=1, bias=True, dilation=1, padding_mode="zeros", device=None, dtype=None):
        super().__init__()
        if groups != 1 or dilation != 1:
            raise NotImplementedError("only groups=1, dilation=1 (all the reference uses)")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride = int(kernel_size), int(stride)
        self.padding, self.output_padding = int(padding), int(output_padding)
        self.causal_crop = 0  # set by CausalConvTranspose1d
        ref = nn.ConvTranspose1d(in_channels, out_channels, self.kernel_size, stride, bias=bias)
        _wn_init(self, ref.weight, ref.bias)
        self._cache = {}  # cfg -> _DeviceCache (the shape table's tile and narrow-launch tiles)

    def phase_cfg(self, B: int = 0, Tin: int = 0) -> int:
        """Tile of the per-phase convs (Kp taps, stride 1); with the launch's B and input length, the narrow-launch
        choice (bc_conv1d_select_cfg_n: each phase writes about Tin columns per clip)."""
        lib = L.load()
        Kp = lib.bc_convT1d_phase_taps(self.kernel_size, self.stride)
        cfg = L.conv_cfg(self.out_channels, self.in_channels, Kp, 1, 1, L.precision_mode())
        if B > 0 and 0 < Tin <= 128:
            n = lib.bc_conv1d_select_cfg_n(self.out_channels, self.in_channels, Kp, 1, 1, L.precision_mode(), B, Tin)
            cfg = n if n >= 0 else cfg
        return cfg

    def prepared(self, device, cfg: Optional[int] = None):
        cfg = self.phase_cfg() if cfg is None else cfg

        def build():
            w = self.folded_weight()  # (Cin, Cout, K)
            Cin, Cout, K = w.shape
            s = self.stride
            lib = L.load()
            Kp = lib.bc_convT1d_phase_taps(K, s)
            n = L.checked_size(lib.bc_conv1d_packed_floats(Cout, Cin, Kp, cfg),
                               f"bc_conv1d_packed_floats({Cout}, {Cin}, {Kp}, cfg {cfg})")
            wt = w.permute(1, 0, 2).contiguous()  # (Cout, Cin, K)
            phases = []
            for r in range(s):
                wr = torch.zeros(Cout, Cin, Kp, dtype=torch.float32)
                for jp in range(Kp):
                    k = r + s * (Kp - 1 - jp)
                    if k < K:
                        wr[:, :, jp] = wt[:, :, k]
                packed = np.empty(n, dtype=np.float32)
                L.call("bc_conv1d_pack", wr.contiguous().numpy().ctypes.data, packed.ctypes.data, Cout, Cin, Kp, cfg)
                phases.append(torch.from_numpy(packed).to(device))
            bias = _cpu(self.bias).contiguous().to(device) if self.bias is not None else None
            return phases, L.ptr_array([p.data_ptr() for p in phases]), bias, cfg
        return self._cache.setdefault(cfg, _DeviceCache()).get(_pkey(*self._params()) + (str(device), cfg), build)

    def out_len(self, T: int) -> int:
        full = (T - 1) * self.stride - 2 * self.padding + self.kernel_size + self.output_padding
        return full - self.causal_crop

    def run(self, x, out_snake=None, dual: bool = False):
        x = _as_input(x)
        B, Cin, T = x.shape
        if Cin != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {Cin}")
        phases, _, bias, cfg = self.prepared(x.device, self.phase_cfg(B, T))
        Tout = self.out_len(T)
        if Tout <= 0:
            raise ValueError(f"input length {T} too short for this transposed convolution")
        sa, sb = _epilogue_args(out_snake, dual)
        out = ops.load().conv_transpose1d(x, phases, bias, sa, sb, self.out_channels, Tout, self.kernel_size,
                                          self.stride, self.padding, cfg, dual)
        return (out[0], out[1]) if dual else out[0]

    def forward(self, x):
        return self.run(x)


class CausalConvTranspose1d(nn.Module):
    """vq/module.py:50-57: transposed conv without padding, last `stride` samples cropped."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, bias=True, device=None, dtype=None):
        super().__init__()
        self.conv = ConvTranspose1dWN(in_channels, out_channels, kernel_size, stride, bias=bias)
        self.stride = stride
        self.conv.causal_crop = stride

    def run(self, x, out_snake=None, dual: bool = False):
        return self.conv.run(x, out_snake, dual)

    def forward(self, x):
        return self.conv.run(x)


def WNConvTranspose1d(*args, causal=False, **kwargs):
    """vq/module.py:67-72."""
    if causal:
        return CausalConvTranspose1d(*args, **kwargs)
    return ConvTranspose1dWN(*args, **kwargs)
