"""BigCodec modules with the reference's constructor signatures and state_dict layout, computing on
the gfx950 HIP kernels of libbigcodec_hip.so.

Drop-in surface: every class here has the same name, constructor arguments,
parameter/buffer names and forward signature as its counterpart in the reference's vq/ package,
so a reference state_dict loads strictly and the callers (lightning_module.py:266-285,
extract_indices.py:353-363, inference_full.py:557-561) work unchanged.  Forward passes run only
on device tensors (fp32); there is no CPU / eager fallback — a CPU input raises.

Composite modules run fused kernels: the Snake of every Activation1d is applied inside the input
staging of the conv that follows it, and ResidualUnit's skip add is the second conv's epilogue.
Folded weights (weight-norm g*v/||v|| evaluated by torch._weight_norm on the CPU, bit-identical
to the reference's per-forward recomputation) are packed once per parameter version and cached
on the device.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn
from torch.nn import Parameter

from . import _lib as L

__all__ = [
    "SnakeBeta", "Snake", "Activation1d", "UpSample1d", "DownSample1d", "LowPassFilter1d",
    "kaiser_sinc_filter1d", "WNConv1d", "WNConvTranspose1d", "CausalConv1d", "CausalConvTranspose1d",
    "Conv1dWN", "ConvTranspose1dWN", "ResidualUnit", "EncoderBlock", "DecoderBlock", "LSTM", "ResLSTM",
    "FactorizedVectorQuantize", "ResidualVQ",
]


# ------------------------------------------------------------------------------------------------
# helpers
# ------------------------------------------------------------------------------------------------
def _as_input(x: torch.Tensor) -> torch.Tensor:
    if not isinstance(x, torch.Tensor) or not x.is_cuda:
        raise L.BigCodecLibraryError(
            "BigCodec HIP modules compute on the GPU only: move the module and its input to a HIP "
            "device (there is no CPU fallback)")
    if x.dtype != torch.float32:
        raise TypeError(f"BigCodec HIP modules compute in fp32 (got {x.dtype})")
    return x if x.is_contiguous() else x.contiguous()


def _pkey(*params) -> tuple:
    """Cache key: identity, in-place version and device of every source parameter."""
    return tuple((id(p), p._version, str(p.device)) if p is not None else None for p in params)


class _DeviceCache:
    def __init__(self):
        self.key = None
        self.val = None

    def get(self, key, build):
        if self.key != key:
            self.val = build()
            self.key = key
        return self.val


def _cpu(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to("cpu", torch.float32)


# ------------------------------------------------------------------------------------------------
# activations  (vq/activations.py, vq/alias_free_torch/)
# ------------------------------------------------------------------------------------------------
class SnakeBeta(nn.Module):
    """vq/activations.py:62-119.  forward = x + 1/(beta+1e-9) * sin(x*alpha)^2 (log-scale params
    exponentiated).  Per-channel coefficients are evaluated once on the host with the reference's
    own torch expressions; the per-element part runs on the GPU."""

    def __init__(self, in_features, alpha=1.0, alpha_trainable=True, alpha_logscale=False):
        super().__init__()
        self.in_features = in_features
        self.alpha_logscale = alpha_logscale
        if alpha_logscale:
            self.alpha = Parameter(torch.zeros(in_features) * alpha)
            self.beta = Parameter(torch.zeros(in_features) * alpha)
        else:
            self.alpha = Parameter(torch.ones(in_features) * alpha)
            self.beta = Parameter(torch.ones(in_features) * alpha)
        self.alpha.requires_grad = alpha_trainable
        self.beta.requires_grad = alpha_trainable
        self.no_div_by_zero = 0.000000001
        self._cache = _DeviceCache()

    def _host_coeffs(self):
        alpha = _cpu(self.alpha)
        beta = _cpu(self.beta)
        if self.alpha_logscale:
            alpha = torch.exp(alpha)
            beta = torch.exp(beta)
        return alpha, 1.0 / (beta + self.no_div_by_zero)

    def coeffs(self, device):
        """(alpha_exp, inv_beta) fp32 device tensors of shape (C,)."""
        def build():
            a, ib = self._host_coeffs()
            return a.contiguous().to(device), ib.contiguous().to(device)
        return self._cache.get(_pkey(self.alpha, self.beta) + (str(device),), build)

    def forward(self, x):
        x = _as_input(x)
        a, ib = self.coeffs(x.device)
        y = torch.empty_like(x)
        B, C, T = x.shape
        L.call("bc_snake_fwd", x.data_ptr(), a.data_ptr(), ib.data_ptr(), y.data_ptr(), B, C, T,
               L.stream_of(x))
        return y


class Snake(SnakeBeta):
    """vq/activations.py:9-59 (unused by the shipped models): x + 1/(alpha+1e-9) * sin(x*alpha)^2."""

    def __init__(self, in_features, alpha=1.0, alpha_trainable=True, alpha_logscale=False):
        nn.Module.__init__(self)
        self.in_features = in_features
        self.alpha_logscale = alpha_logscale
        if alpha_logscale:
            self.alpha = Parameter(torch.zeros(in_features) * alpha)
        else:
            self.alpha = Parameter(torch.ones(in_features) * alpha)
        self.alpha.requires_grad = alpha_trainable
        self.no_div_by_zero = 0.000000001
        self._cache = _DeviceCache()

    def _host_coeffs(self):
        alpha = _cpu(self.alpha)
        if self.alpha_logscale:
            alpha = torch.exp(alpha)
        return alpha, 1.0 / (alpha + self.no_div_by_zero)

    def coeffs(self, device):
        def build():
            a, ib = self._host_coeffs()
            return a.contiguous().to(device), ib.contiguous().to(device)
        return self._cache.get(_pkey(self.alpha) + (str(device),), build)


def kaiser_sinc_filter1d(cutoff, half_width, kernel_size):
    """vq/alias_free_torch/filter.py:28-57 (init-time constant; returns (1,1,kernel_size))."""
    even = kernel_size % 2 == 0
    half_size = kernel_size // 2
    delta_f = 4 * half_width
    A = 2.285 * (half_size - 1) * math.pi * delta_f + 7.95
    if A > 50.0:
        beta = 0.1102 * (A - 8.7)
    elif A >= 21.0:
        beta = 0.5842 * (A - 21) ** 0.4 + 0.07886 * (A - 21.0)
    else:
        beta = 0.0
    window = torch.kaiser_window(kernel_size, beta=beta, periodic=False)
    if even:
        time = torch.arange(-half_size, half_size) + 0.5
    else:
        time = torch.arange(kernel_size) - half_size
    if cutoff == 0:
        filter_ = torch.zeros_like(time)
    else:
        filter_ = 2 * cutoff * window * torch.sinc(2 * cutoff * time)
        filter_ /= filter_.sum()
    return filter_.view(1, 1, kernel_size)


class UpSample1d(nn.Module):
    """vq/alias_free_torch/resample.py:10-33 (parameter holder; the math runs in bc_aa_snake_fwd)."""

    def __init__(self, ratio=2, kernel_size=None):
        super().__init__()
        self.ratio = ratio
        self.kernel_size = int(6 * ratio // 2) * 2 if kernel_size is None else kernel_size
        self.stride = ratio
        self.pad = self.kernel_size // ratio - 1
        self.pad_left = self.pad * self.stride + (self.kernel_size - self.stride) // 2
        self.pad_right = self.pad * self.stride + (self.kernel_size - self.stride + 1) // 2
        self.register_buffer("filter", kaiser_sinc_filter1d(0.5 / ratio, 0.6 / ratio, self.kernel_size))


class LowPassFilter1d(nn.Module):
    """vq/alias_free_torch/filter.py:60-95 (parameter holder)."""

    def __init__(self, cutoff=0.5, half_width=0.6, stride: int = 1, padding: bool = True,
                 padding_mode: str = "replicate", kernel_size: int = 12):
        super().__init__()
        if cutoff < -0.0:
            raise ValueError("Minimum cutoff must be larger than zero.")
        if cutoff > 0.5:
            raise ValueError("A cutoff above 0.5 does not make sense.")
        self.kernel_size = kernel_size
        self.even = kernel_size % 2 == 0
        self.pad_left = kernel_size // 2 - int(self.even)
        self.pad_right = kernel_size // 2
        self.stride = stride
        self.padding = padding
        self.padding_mode = padding_mode
        self.register_buffer("filter", kaiser_sinc_filter1d(cutoff, half_width, kernel_size))


class DownSample1d(nn.Module):
    """vq/alias_free_torch/resample.py:36-49 (parameter holder)."""

    def __init__(self, ratio=2, kernel_size=None):
        super().__init__()
        self.ratio = ratio
        self.kernel_size = int(6 * ratio // 2) * 2 if kernel_size is None else kernel_size
        self.lowpass = LowPassFilter1d(cutoff=0.5 / ratio, half_width=0.6 / ratio, stride=ratio,
                                       kernel_size=self.kernel_size)


class Activation1d(nn.Module):
    """vq/alias_free_torch/act.py:7-32.  Without antialias the Snake alone; with antialias the fused
    up(2x, 12 taps) -> Snake -> down(2x, 12 taps) kernel."""

    def __init__(self, activation, antialias: bool = False, up_ratio: int = 2, down_ratio: int = 2,
                 up_kernel_size: int = 12, down_kernel_size: int = 12):
        super().__init__()
        self.antialias = antialias
        self.up_ratio = up_ratio
        self.down_ratio = down_ratio
        self.act = activation
        if antialias:
            if (up_ratio, down_ratio, up_kernel_size, down_kernel_size) != (2, 2, 12, 12):
                raise NotImplementedError("anti-aliased Activation1d is implemented for ratio 2, 12 taps "
                                          "(the only configuration the reference builds)")
            self.upsample = UpSample1d(up_ratio, up_kernel_size)
            self.downsample = DownSample1d(down_ratio, down_kernel_size)
        self._fcache = _DeviceCache()

    def filters(self, device):
        f_up, f_dn = self.upsample.filter, self.downsample.lowpass.filter

        def build():
            return (_cpu(f_up).reshape(-1).contiguous().to(device),
                    _cpu(f_dn).reshape(-1).contiguous().to(device))
        return self._fcache.get(_pkey(f_up, f_dn) + (str(device),), build)

    def snake_coeffs(self, device):
        """Coefficients for fusing this activation into the next conv (None if not fusable)."""
        if self.antialias:
            return None
        return self.act.coeffs(device)

    def forward(self, x):
        if not self.antialias:
            return self.act(x)
        x = _as_input(x)
        a, ib = self.act.coeffs(x.device)
        fu, fd = self.filters(x.device)
        y = torch.empty_like(x)
        B, C, T = x.shape
        L.call("bc_aa_snake_fwd", x.data_ptr(), a.data_ptr(), ib.data_ptr(), fu.data_ptr(),
               fd.data_ptr(), y.data_ptr(), B, C, T, L.stream_of(x))
        return y


def run_activation_then(act: Activation1d, x: torch.Tensor):
    """Return (input for the next conv, snake coefficients to fuse or None)."""
    co = act.snake_coeffs(x.device)
    if co is not None:
        return x, co
    return act(x), None


# ------------------------------------------------------------------------------------------------
# convolutions  (vq/module.py:11-72)
# ------------------------------------------------------------------------------------------------
class Conv1dWN(nn.Module):
    """weight_norm(nn.Conv1d(...)) with the same parameter names (bias, weight_g, weight_v) and the
    same constructor signature as nn.Conv1d (groups=1, padding_mode='zeros')."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, bias=True, padding_mode="zeros", device=None, dtype=None):
        super().__init__()
        if groups != 1 or padding_mode != "zeros":
            raise NotImplementedError("only groups=1, padding_mode='zeros' (all the reference uses)")
        if isinstance(padding, str):
            raise NotImplementedError("string padding is not used by the reference")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = int(kernel_size[0] if isinstance(kernel_size, (tuple, list)) else kernel_size)
        self.stride = int(stride[0] if isinstance(stride, (tuple, list)) else stride)
        self.padding = int(padding[0] if isinstance(padding, (tuple, list)) else padding)
        self.dilation = int(dilation[0] if isinstance(dilation, (tuple, list)) else dilation)
        self.causal_pad: Optional[int] = None  # set by CausalConv1d
        ref = nn.Conv1d(in_channels, out_channels, self.kernel_size, bias=bias)  # default init
        if bias:
            self.bias = Parameter(ref.bias.detach().clone().zero_())
        else:
            self.register_parameter("bias", None)
        v = ref.weight.detach().clone()
        self.weight_g = Parameter(torch.linalg.vector_norm(v.reshape(v.shape[0], -1), dim=1).reshape(-1, 1, 1))
        self.weight_v = Parameter(v)
        self._cache = _DeviceCache()

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

    def prepared(self, device):
        def build():
            w = self.folded_weight().contiguous()
            Cout, Cin, K = w.shape
            cfg = L.load().bc_conv1d_select_cfg(Cout, Cin)
            n = L.load().bc_conv1d_packed_floats(Cout, Cin, K, cfg)
            packed = np.empty(n, dtype=np.float32)
            wn = w.numpy()
            L.call("bc_conv1d_pack", wn.ctypes.data, packed.ctypes.data, Cout, Cin, K, cfg)
            bias = _cpu(self.bias).contiguous().to(device) if self.bias is not None else None
            return torch.from_numpy(packed).to(device), bias, cfg
        return self._cache.get(_pkey(*self._params()) + (str(device),), build)

    def out_len(self, T: int) -> int:
        pl = self.pad_left()
        pr = 0 if self.causal_pad is not None else self.padding
        return (T + pl + pr - self.dilation * (self.kernel_size - 1) - 1) // self.stride + 1

    def pad_left(self) -> int:
        return self.causal_pad if self.causal_pad is not None else self.padding

    def run(self, x, snake=None, residual=None, epilogue: int = 0):
        x = _as_input(x)
        B, Cin, T = x.shape
        if Cin != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {Cin}")
        wp, bias, cfg = self.prepared(x.device)
        Tout = self.out_len(T)
        if Tout <= 0:
            raise ValueError(f"input length {T} too short for this convolution")
        y = torch.empty((B, self.out_channels, Tout), device=x.device, dtype=torch.float32)
        if residual is not None:
            residual = _as_input(residual)
            if residual.shape != y.shape:
                raise ValueError(f"residual shape {tuple(residual.shape)} != output {tuple(y.shape)}")
        sa, sb = snake if snake is not None else (None, None)
        tm = L.active_timer()
        ev = tm.begin() if tm is not None else None
        L.call("bc_conv1d_fwd", x.data_ptr(), wp.data_ptr(), L.ptr(bias), L.ptr(sa), L.ptr(sb),
               L.ptr(residual), y.data_ptr(), B, Cin, T, self.out_channels, Tout, self.kernel_size,
               self.stride, self.dilation, self.pad_left(), epilogue, cfg, L.stream_of(x))
        if tm is not None:
            flops = 2.0 * B * self.out_channels * Cin * self.kernel_size * Tout
            nbytes = 4.0 * (x.numel() + y.numel() * (2 if residual is not None else 1))
            tm.end(ev, L.conv_kernel_name(cfg, snake is not None), flops, nbytes)
        return y

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

    def run(self, x, snake=None, residual=None, epilogue: int = 0):
        return self.conv.run(x, snake, residual, epilogue)

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


class ConvTranspose1dWN(nn.Module):
    """weight_norm(nn.ConvTranspose1d(...)): weight_v (Cin, Cout, K), weight_g (Cin, 1, 1) — the
    norm runs over dim 0 = INPUT channels — and bias (Cout)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0,
                 groups=1, bias=True, dilation=1, padding_mode="zeros", device=None, dtype=None):
        super().__init__()
        if groups != 1 or dilation != 1:
            raise NotImplementedError("only groups=1, dilation=1 (all the reference uses)")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = int(kernel_size)
        self.stride = int(stride)
        self.padding = int(padding)
        self.output_padding = int(output_padding)
        self.causal_crop = 0  # set by CausalConvTranspose1d
        ref = nn.ConvTranspose1d(in_channels, out_channels, self.kernel_size, stride, bias=bias)
        if bias:
            self.bias = Parameter(ref.bias.detach().clone())
        else:
            self.register_parameter("bias", None)
        v = ref.weight.detach().clone()
        self.weight_g = Parameter(torch.linalg.vector_norm(v.reshape(v.shape[0], -1), dim=1).reshape(-1, 1, 1))
        self.weight_v = Parameter(v)
        self._cache = _DeviceCache()

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

    def prepared(self, device):
        def build():
            w = self.folded_weight()  # (Cin, Cout, K)
            Cin, Cout, K = w.shape
            s = self.stride
            lib = L.load()
            Kp = lib.bc_convT1d_phase_taps(K, s)
            cfg = lib.bc_conv1d_select_cfg(Cout, Cin)
            n = lib.bc_conv1d_packed_floats(Cout, Cin, Kp, cfg)
            wt = w.permute(1, 0, 2).contiguous()  # (Cout, Cin, K)
            phases = []
            for r in range(s):
                wr = torch.zeros(Cout, Cin, Kp, dtype=torch.float32)
                for jp in range(Kp):
                    k = r + s * (Kp - 1 - jp)
                    if k < K:
                        wr[:, :, jp] = wt[:, :, k]
                packed = np.empty(n, dtype=np.float32)
                wrn = wr.contiguous().numpy()
                L.call("bc_conv1d_pack", wrn.ctypes.data, packed.ctypes.data, Cout, Cin, Kp, cfg)
                phases.append(torch.from_numpy(packed).to(device))
            bias = _cpu(self.bias).contiguous().to(device) if self.bias is not None else None
            return phases, L.ptr_array([p.data_ptr() for p in phases]), bias, cfg
        return self._cache.get(_pkey(*self._params()) + (str(device),), build)

    def out_len(self, T: int) -> int:
        full = (T - 1) * self.stride - 2 * self.padding + self.kernel_size + self.output_padding
        return full - self.causal_crop

    def run(self, x, snake=None):
        x = _as_input(x)
        B, Cin, T = x.shape
        if Cin != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {Cin}")
        _, parr, bias, cfg = self.prepared(x.device)
        Tout = self.out_len(T)
        y = torch.empty((B, self.out_channels, Tout), device=x.device, dtype=torch.float32)
        sa, sb = snake if snake is not None else (None, None)
        L.call("bc_convT1d_fwd", x.data_ptr(), parr, L.ptr(bias), L.ptr(sa), L.ptr(sb), y.data_ptr(), B,
               Cin, T, self.out_channels, Tout, self.kernel_size, self.stride, self.padding, cfg,
               L.stream_of(x))
        return y

    def forward(self, x):
        return self.run(x)


class CausalConvTranspose1d(nn.Module):
    """vq/module.py:50-57: transposed conv without padding, last `stride` samples cropped."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, bias=True, device=None, dtype=None):
        super().__init__()
        self.conv = ConvTranspose1dWN(in_channels, out_channels, kernel_size, stride, bias=bias)
        self.stride = stride
        self.conv.causal_crop = stride

    def run(self, x, snake=None):
        return self.conv.run(x, snake)

    def forward(self, x):
        return self.conv.run(x)


def WNConvTranspose1d(*args, causal=False, **kwargs):
    """vq/module.py:67-72."""
    if causal:
        return CausalConvTranspose1d(*args, **kwargs)
    return ConvTranspose1dWN(*args, **kwargs)


def _conv_of(m) -> Conv1dWN:
    return m.conv if isinstance(m, CausalConv1d) else m


# ------------------------------------------------------------------------------------------------
# blocks  (vq/module.py:74-167)
# ------------------------------------------------------------------------------------------------
class ResidualUnit(nn.Module):
    """vq/module.py:74-89: x + conv1(snake(conv7_d(snake(x)))) as two fused launches:
    conv7 with the first Snake in its prologue, conv1 with the second Snake in its prologue and
    the skip add in its epilogue."""

    def __init__(self, dim: int = 16, dilation: int = 1, causal: bool = False, antialias: bool = False):
        super().__init__()
        pad = 0 if causal else ((7 - 1) * dilation) // 2
        self.block = nn.Sequential(
            Activation1d(activation=SnakeBeta(dim, alpha_logscale=True), antialias=antialias),
            WNConv1d(dim, dim, kernel_size=7, dilation=dilation, padding=pad, causal=causal),
            Activation1d(activation=SnakeBeta(dim, alpha_logscale=True), antialias=antialias),
            WNConv1d(dim, dim, kernel_size=1),
        )

    def forward(self, x):
        x = _as_input(x)
        h, co = run_activation_then(self.block[0], x)
        h = self.block[1].run(h, snake=co)
        h, co = run_activation_then(self.block[2], h)
        return self.block[3].run(h, snake=co, residual=x)


class EncoderBlock(nn.Module):
    """vq/module.py:91-113: 3 ResidualUnits -> Snake -> strided conv (k=2s) C/2 -> C."""

    def __init__(self, dim: int = 16, stride: int = 1, dilations=(1, 3, 9), causal: bool = False,
                 antialias: bool = False):
        super().__init__()
        runits = [ResidualUnit(dim // 2, dilation=d, causal=causal, antialias=antialias) for d in dilations]
        pad = 0 if causal else (stride // 2 + stride % 2 if stride != 1 else 0)
        self.block = nn.Sequential(
            *runits,
            Activation1d(activation=SnakeBeta(dim // 2, alpha_logscale=True), antialias=antialias),
            WNConv1d(dim // 2, dim, kernel_size=2 * stride if stride != 1 else 1, stride=stride,
                     padding=pad, causal=causal),
        )

    def forward(self, x):
        n = len(self.block)
        for i in range(n - 2):
            x = self.block[i](x)
        h, co = run_activation_then(self.block[n - 2], x)
        return self.block[n - 1].run(h, snake=co)


class DecoderBlock(nn.Module):
    """vq/module.py:115-141: Snake -> transposed conv (k=2s) -> 3 ResidualUnits."""

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
            WNConvTranspose1d(input_dim, output_dim, kernel_size=2 * stride if stride != 1 else 1,
                              stride=stride, causal=causal, **tconv_kwargs),
        )
        self.block.extend([ResidualUnit(output_dim, dilation=d, causal=causal, antialias=antialias)
                           for d in dilations])

    def forward(self, x):
        x = _as_input(x)
        h, co = run_activation_then(self.block[0], x)
        x = self.block[1].run(h, snake=co)
        for i in range(2, len(self.block)):
            x = self.block[i](x)
        return x


class LSTM(nn.Module):
    """Parameter container with torch.nn.LSTM's names (weight_ih_l{k}, weight_hh_l{k}, bias_ih_l{k},
    bias_hh_l{k}; batch_first) so reference checkpoints load; the recurrence runs in
    bc_reslstm_fwd."""

    def __init__(self, input_size, hidden_size, num_layers=1, bias=True, batch_first=True,
                 dropout=0.0, bidirectional=False):
        super().__init__()
        if bidirectional:
            raise NotImplementedError("bidirectional ResLSTM is not used by any shipped config")
        if not bias or not batch_first or dropout:
            raise NotImplementedError("only bias=True, batch_first=True, dropout=0")
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.batch_first, self.bidirectional = batch_first, bidirectional
        ref = nn.LSTM(input_size, hidden_size, num_layers, batch_first=True)  # torch's default init
        for name, p in ref.named_parameters():
            setattr(self, name, Parameter(p.detach().clone()))
        self._cache = _DeviceCache()

    def _plist(self):
        out = []
        for l in range(self.num_layers):
            out += [getattr(self, f"weight_ih_l{l}"), getattr(self, f"weight_hh_l{l}"),
                    getattr(self, f"bias_ih_l{l}"), getattr(self, f"bias_hh_l{l}")]
        return out

    def prepared(self, device):
        def build():
            lib = L.load()
            H = self.hidden_size
            if self.input_size != H:
                raise NotImplementedError("ResLSTM requires input_size == hidden_size")
            cfg = lib.bc_conv1d_select_cfg(4 * H, H)
            wih, whh, bias = [], [], []
            for l in range(self.num_layers):
                w = _cpu(getattr(self, f"weight_ih_l{l}")).contiguous()
                n = lib.bc_conv1d_packed_floats(4 * H, H, 1, cfg)
                packed = np.empty(n, dtype=np.float32)
                L.call("bc_conv1d_pack", w.numpy().ctypes.data, packed.ctypes.data, 4 * H, H, 1, cfg)
                wih.append(torch.from_numpy(packed).to(device))
                w = _cpu(getattr(self, f"weight_hh_l{l}")).contiguous()
                packed = np.empty(lib.bc_lstm_hh_packed_floats(H), dtype=np.float32)
                L.call("bc_lstm_pack_hh", w.numpy().ctypes.data, packed.ctypes.data, H)
                whh.append(torch.from_numpy(packed).to(device))
                b = _cpu(getattr(self, f"bias_ih_l{l}")) + _cpu(getattr(self, f"bias_hh_l{l}"))
                bias.append(b.contiguous().to(device))
            arrs = (L.ptr_array([t.data_ptr() for t in wih]), L.ptr_array([t.data_ptr() for t in bias]),
                    L.ptr_array([t.data_ptr() for t in whh]))
            return (wih, whh, bias), arrs
        return self._cache.get(_pkey(*self._plist()) + (str(device),), build)


class ResLSTM(nn.Module):
    """vq/module.py:143-167: y = LSTM(x^T)^T + x for x (B, F, T)."""

    def __init__(self, dimension: int, num_layers: int = 2, bidirectional: bool = False, skip: bool = True):
        super().__init__()
        if not skip:
            raise NotImplementedError("ResLSTM(skip=False) is not used by the reference models")
        self.skip = skip
        self.lstm = LSTM(dimension, dimension if not bidirectional else dimension // 2, num_layers,
                         batch_first=True, bidirectional=bidirectional)

    def forward(self, x):
        x = _as_input(x)
        B, H, T = x.shape
        _, (pwih, pbias, pwhh) = self.lstm.prepared(x.device)
        lib = L.load()
        ws = torch.empty(int(lib.bc_lstm_workspace_floats(B, H, T)), device=x.device, dtype=torch.float32)
        y = torch.empty_like(x)
        L.call("bc_reslstm_fwd", x.data_ptr(), y.data_ptr(), B, H, T, self.lstm.num_layers, pwih, pbias,
               pwhh, ws.data_ptr(), L.stream_of(x))
        return y


# ------------------------------------------------------------------------------------------------
# quantizer  (vq/factorized_vector_quantize.py, vq/residual_vq.py)
# ------------------------------------------------------------------------------------------------
class LinearWN(nn.Module):
    """weight_norm(nn.Linear(in, out)): weight_g (out, 1), weight_v (out, in), bias (out)."""

    def __init__(self, in_features, out_features):
        super().__init__()
        ref = nn.Linear(in_features, out_features)
        self.in_features, self.out_features = in_features, out_features
        self.bias = Parameter(ref.bias.detach().clone())
        v = ref.weight.detach().clone()
        self.weight_g = Parameter(torch.linalg.vector_norm(v, dim=1).reshape(-1, 1))
        self.weight_v = Parameter(v)

    def folded_weight(self):
        if "weight" in self._parameters:
            return _cpu(self._parameters["weight"])
        return torch._weight_norm(_cpu(self.weight_v), _cpu(self.weight_g), 0)

    def _params(self):
        if "weight" in self._parameters:
            return (self._parameters["weight"], self.bias)
        return (self.weight_g, self.weight_v, self.bias)


class _Embedding(nn.Module):
    """nn.Embedding parameter holder (`weight`)."""

    def __init__(self, num_embeddings, embedding_dim):
        super().__init__()
        self.num_embeddings, self.embedding_dim = num_embeddings, embedding_dim
        self.weight = Parameter(torch.randn(num_embeddings, embedding_dim))


class FactorizedVectorQuantize(nn.Module):
    """vq/factorized_vector_quantize.py:10-108 (eval forward)."""

    def __init__(self, dim, codebook_size, codebook_dim, commitment, **kwargs):
        super().__init__()
        self.codebook_size = codebook_size
        self.codebook_dim = codebook_dim
        self.commitment = commitment
        self.dim = dim
        if codebook_dim != 8:
            raise NotImplementedError("the HIP VQ kernels are built for codebook_dim == 8 (every config)")
        if dim != codebook_dim:
            self.in_proj = LinearWN(dim, codebook_dim)
            self.out_proj = LinearWN(codebook_dim, dim)
        else:
            raise NotImplementedError("dim == codebook_dim (identity projections) is not used by the reference")
        self._codebook = _Embedding(codebook_size, codebook_dim)
        self._cache = _DeviceCache()

    @property
    def codebook(self):
        return self._codebook

    def prepared(self, device):
        cbw = self._codebook.weight

        def build():
            lib = L.load()
            cb = _cpu(cbw).contiguous().to(device)
            cbn = torch.empty_like(cb)
            csq = torch.empty(cb.shape[0], device=device, dtype=torch.float32)
            stream = torch.cuda.current_stream(device).cuda_stream
            L.check(lib.bc_vq_prepare_codebook(cb.data_ptr(), cbn.data_ptr(), csq.data_ptr(), cb.shape[0],
                                               self.codebook_dim, stream), "bc_vq_prepare_codebook")
            w_in = self.in_proj.folded_weight().contiguous().to(device)
            b_in = _cpu(self.in_proj.bias).contiguous().to(device)
            w_out = self.out_proj.folded_weight().contiguous().to(device)
            b_out = _cpu(self.out_proj.bias).contiguous().to(device)
            return cb, cbn, csq, w_in, b_in, w_out, b_out
        key = _pkey(cbw, *self.in_proj._params(), *self.out_proj._params()) + (str(device),)
        return self._cache.get(key, build)

    def quantize_into(self, z, idx_out, post_out=None, ze_out=None):
        """Run the fused kernel; idx_out (B,T) int64 view, post_out (B,D,T) or None."""
        B, D, T = z.shape
        cb, cbn, csq, w_in, b_in, w_out, b_out = self.prepared(z.device)
        L.call("bc_vq_fwd", z.data_ptr(), w_in.data_ptr(), b_in.data_ptr(), cb.data_ptr(), cbn.data_ptr(),
               csq.data_ptr(), w_out.data_ptr(), b_out.data_ptr(), idx_out.data_ptr(), L.ptr(ze_out),
               L.ptr(post_out), B, D, T, self.codebook_size, self.codebook_dim, L.stream_of(z))

    def forward(self, z):
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("training-mode VQ (losses / straight-through gradients) is out of "
                                      "scope of the HIP inference path; call .eval()")
        z = _as_input(z)
        B, D, T = z.shape
        if D != self.dim:
            raise ValueError(f"expected {self.dim} channels, got {D}")
        idx = torch.empty((B, T), device=z.device, dtype=torch.int64)
        post = torch.empty_like(z)
        self.quantize_into(z, idx, post)
        commit_loss = torch.zeros(B, device=z.device)
        return post, idx, commit_loss

    def vq2emb(self, vq, proj=True):
        """indices (...) int64 -> out_proj(codebook[indices]) (..., D)  (:78-81)."""
        if not vq.is_cuda:
            raise L.BigCodecLibraryError("vq2emb takes device index tensors")
        if vq.dtype != torch.int64:
            raise TypeError("indices must be int64")
        vq = vq.contiguous()
        return self._vq2emb_into_strided(vq.unsqueeze(-1), 0, 1, None, proj, accumulate=False)

    def get_emb(self):
        return self.codebook.weight

    def embed_code(self, embed_id):
        return self.vq2emb(embed_id, proj=False)

    def decode_code(self, embed_id):
        return self.embed_code(embed_id).transpose(1, 2)


class ResidualVQ(nn.Module):
    """vq/residual_vq.py:6-53."""

    def __init__(self, *, num_quantizers, codebook_size, **kwargs):
        super().__init__()
        if isinstance(codebook_size, int):
            codebook_size = [codebook_size] * num_quantizers
        kwargs = {k: v for k, v in kwargs.items() if k in ("dim", "codebook_dim", "commitment")}
        self.layers = nn.ModuleList([FactorizedVectorQuantize(codebook_size=size, **kwargs)
                                     for size in codebook_size])
        self.num_quantizers = num_quantizers

    def quantize(self, x, idx_out=None, with_post=True):
        """Fused forward; idx_out optional preallocated (Nq, B, T) int64."""
        x = _as_input(x)
        B, D, T = x.shape
        nq = len(self.layers)
        if idx_out is None:
            idx_out = torch.empty((nq, B, T), device=x.device, dtype=torch.int64)
        if nq == 1:
            post = torch.empty_like(x) if with_post else None
            self.layers[0].quantize_into(x, idx_out[0], post)
            return post, idx_out
        residual = x.clone()
        out = torch.empty_like(x)
        q = torch.empty_like(x)
        stream = L.stream_of(x)
        for i, layer in enumerate(self.layers):
            layer.quantize_into(residual, idx_out[i], q)
            L.call("bc_rvq_update", residual.data_ptr(), out.data_ptr(), q.data_ptr(), residual.numel(),
                   int(i == 0), stream)
        return out, idx_out

    def forward(self, x):
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("training-mode VQ is out of scope of the HIP inference path; call .eval()")
        quantized_out, all_indices = self.quantize(x)
        all_losses = torch.zeros(len(self.layers), device=quantized_out.device)
        return quantized_out, all_indices, all_losses

    def vq2emb(self, vq, proj=True):
        # vq: (B, T, Nq) int64 -> (B, T, D)
        if not vq.is_contiguous():
            raise ValueError("vq2emb expects a contiguous (B, T, num_quantizers) index tensor")
        nq = vq.shape[-1]
        out = None
        for i, layer in enumerate(self.layers[:nq]):
            out = layer._vq2emb_into_strided(vq, i, nq, out, proj, accumulate=i > 0)
        return out

    def get_emb(self):
        return [layer.get_emb() for layer in self.layers]


def _vq2emb_into_strided(self, vq, i, nq, out, proj, accumulate):
    """vq: contiguous (..., nq) int64; uses column i (element stride nq)."""
    if not vq.is_cuda or vq.dtype != torch.int64 or not vq.is_contiguous():
        raise ValueError("vq2emb expects a contiguous int64 device tensor")
    cb, _, _, _, _, w_out, b_out = self.prepared(vq.device)
    D = self.dim if proj else self.codebook_dim
    shape = tuple(vq.shape[:-1])
    N = int(np.prod(shape))
    if out is None:
        out = torch.empty(shape + (D,), device=vq.device, dtype=torch.float32)
    base = vq.data_ptr() + i * vq.element_size()
    L.call("bc_vq2emb", base, nq, cb.data_ptr(), L.ptr(w_out if proj else None), L.ptr(b_out if proj else None),
           out.data_ptr(), N, D, self.codebook_size, self.codebook_dim, int(accumulate), L.stream_of(out))
    return out


FactorizedVectorQuantize._vq2emb_into_strided = _vq2emb_into_strided
