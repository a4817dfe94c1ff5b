"""Activations (vq/activations.py, vq/alias_free_torch/) and the factorized VQ
(vq/factorized_vector_quantize.py, vq/residual_vq.py) with the reference's constructor signatures
and state_dict layout, computing on the gfx950 HIP kernels of libbigcodec_hip.so.

Drop-in surface: every class here, in conv.py and in blocks.py has the same name,
constructor arguments, parameter/buffer names and forward signature as its counterpart in the
reference's vq/ package, so a reference state_dict loads strictly and the callers
(lightning_module.py:266-285, extract_indices.py:353-363, inference_full.py:557-561) work
unchanged.  Forward passes run only on device tensors (fp32); there is no CPU / eager fallback — a
CPU input raises.  Host-side parameter preparation (weight-norm folding with torch._weight_norm on
the CPU, bit-identical to the reference's per-forward recomputation; per-channel Snake
coefficients) happens once per parameter version and is cached on the device.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
from torch.nn import Parameter

from . import _lib as L
from .ops import load as _ops  # torch.ops.bigcodec namespace (loads libbigcodec_ops.so once)

__all__ = [
    "SnakeBeta", "Snake", "Activation1d", "UpSample1d", "DownSample1d", "LowPassFilter1d",
    "kaiser_sinc_filter1d", "LinearWN", "FactorizedVectorQuantize", "ResidualVQ",
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


_ZEROS = {}


def _zeros(n: int, device) -> torch.Tensor:
    """Cached all-zero fp32 device vector (the eval-mode VQ losses): uploaded once, no fill kernel
    per call.  Callers must not write into it."""
    key = (n, str(device))
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros(n).to(device)
    return z


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
        return _ops().snake(x, a, ib)


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


# Adopted, as the reference's vq/alias_free_torch/filter.py:25-27 states for its own copy, from adefossez's
# julius.lowpass.LowPassFilters under the MIT License (https://adefossez.github.io/julius/julius/lowpass.html);
# the reference's filter.py:1-2 credits the alias-free-torch package (junjun3518) under the Apache License 2.0.
# The buffer values must be bit-identical to the reference's (test_oracle_pinned.py), hence the same expression.
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
    up -> Snake -> down kernel (the default 2x / 12 taps on its own kernel, any other ratios and tap
    counts on the general one)."""

    def __init__(self, activation, antialias: bool = False, up_ratio: int = 2, down_ratio: int = 2,
                 up_kernel_size: int = 12, down_kernel_size: int = 12):
        super().__init__()
        self.antialias = antialias
        self.up_ratio = up_ratio
        self.down_ratio = down_ratio
        self.act = activation
        if antialias:
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
        if (self.up_ratio, self.down_ratio, fu.numel(), fd.numel()) == (2, 2, 12, 12):
            return _ops().aa_snake(x, a, ib, fu, fd)
        # other constructor ratios / tap counts (act.py:8-23): the general kernel (bc_aa_snake_fwd_ex)
        return _ops().aa_snake_ex(x, a, ib, fu, fd, self.up_ratio, self.down_ratio)


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
            cb = _cpu(cbw).contiguous().to(device)
            cbn, csq = _ops().vq_prepare_codebook(cb)
            w_in = self.in_proj.folded_weight().contiguous().to(device)
            b_in = _cpu(self.in_proj.bias).contiguous().to(device)
            w_out = self.out_proj.folded_weight().contiguous().to(device)
            b_out = _cpu(self.out_proj.bias).contiguous().to(device)
            return cb, cbn, csq, w_in, b_in, w_out, b_out
        key = _pkey(cbw, *self.in_proj._params(), *self.out_proj._params()) + (str(device),)
        return self._cache.get(key, build)

    def quantize(self, z, want_post: bool = True, want_ze: bool = False):
        """One fused launch (torch.ops.bigcodec.vq): [indices (B, T) int64, z_e (B, 8, T) if want_ze,
        post-VQ out_proj(z_q) (B, D, T) if want_post]."""
        cb, cbn, csq, w_in, b_in, w_out, b_out = self.prepared(z.device)
        return _ops().vq(z, w_in, b_in, cb, cbn, csq, w_out, b_out, want_ze, want_post)

    def forward(self, z):
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("training-mode VQ (losses / straight-through gradients) is out of "
                                      "scope of the HIP inference path; call .eval()")
        z = _as_input(z)
        B, D, T = z.shape
        if D != self.dim:
            raise ValueError(f"expected {self.dim} channels, got {D}")
        idx, post = self.quantize(z)
        commit_loss = _zeros(B, z.device)  # eval: torch.zeros(B) (factorized_vector_quantize.py:66)
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

    def quantize(self, x, with_post=True):
        """Fused forward -> (post-VQ sum (B, D, T) or None, indices (Nq, B, T) int64)."""
        x = _as_input(x)
        nq = len(self.layers)
        if nq == 1:
            res = self.layers[0].quantize(x, want_post=with_post)
            return (res[1] if with_post else None), res[0].unsqueeze(0)
        residual = x.clone()
        out = torch.empty_like(x)
        idx = []
        for i, layer in enumerate(self.layers):
            ind, q = layer.quantize(residual)
            idx.append(ind)
            _ops().rvq_update_(residual, out, q, i == 0)  # residual -= q; out (+)= q (residual_vq.py:31-33)
        return out, torch.stack(idx)

    def forward(self, x):
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("training-mode VQ is out of scope of the HIP inference path; call .eval()")
        quantized_out, all_indices = self.quantize(x)
        all_losses = _zeros(len(self.layers), quantized_out.device)  # stack of zeros(B).mean()
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

    def prepared_stack(self, device):
        """The quantizers' codebooks, folded out_proj weights and biases stacked for bc_vq2emb_ct
        ([Nq][n_codes][8], [Nq][D][8], [Nq][D]); built once per device and parameter version."""
        preps = [layer.prepared(device) for layer in self.layers]
        if len({layer.codebook_size for layer in self.layers}) != 1:
            raise NotImplementedError("bc_vq2emb_ct stacks equal-size codebooks")
        key = tuple(id(t) for p in preps for t in (p[0], p[5], p[6]))
        cached = getattr(self, "_stack_cache", None)
        if cached is None or cached[0] != key:
            cb = torch.stack([p[0] for p in preps]).contiguous()
            w = torch.stack([p[5] for p in preps]).contiguous()
            bb = torch.stack([p[6] for p in preps]).contiguous()
            self._stack_cache = (key, (cb, w, bb))
        return self._stack_cache[1]

    def vq2emb_ct(self, vq):
        """Token -> decoder input in one launch: vq (B, T, Nq) int64 on the device -> (B, D, T) =
        self.vq2emb(vq).transpose(1, 2) (residual_vq.py:42-48 + the caller's transpose before
        codec_decoder.py decoder(x, vq=False)); Nq may be less than num_quantizers, as in vq2emb."""
        if not vq.is_cuda:
            raise L.BigCodecLibraryError("vq2emb_ct takes device index tensors")
        if vq.dtype != torch.int64 or vq.dim() != 3:
            raise TypeError("indices must be an int64 (B, T, num_quantizers) tensor")
        vq = vq.contiguous()
        B, T, nq = vq.shape
        if not 1 <= nq <= len(self.layers):
            raise ValueError(f"{nq} quantizer columns for a {len(self.layers)}-quantizer ResidualVQ")
        cb, w, bb = self.prepared_stack(vq.device)
        return _ops().vq2emb_ct(vq, cb, w, bb)


def _vq2emb_into_strided(self, vq, i, nq, out, proj, accumulate):
    """vq: contiguous (..., nq) int64; uses column i (element stride nq)."""
    if not vq.is_cuda or vq.dtype != torch.int64 or not vq.is_contiguous():
        raise ValueError("vq2emb expects a contiguous int64 device tensor")
    cb, _, _, _, _, w_out, b_out = self.prepared(vq.device)
    if vq.shape[-1] != nq:
        raise ValueError(f"index tensor has {vq.shape[-1]} columns, expected {nq}")
    w, b = (w_out, b_out) if proj else (None, None)
    if out is None or not accumulate:
        return _ops().vq2emb(vq, i, cb, w, b)
    _ops().vq2emb_add_(out, vq, i, cb, w, b)
    return out


FactorizedVectorQuantize._vq2emb_into_strided = _vq2emb_into_strided


class FSQ(nn.Module):
    """The vendored lucidrains FSQ (vq/vector_quantize_pytorch_lucidrains/finite_scalar_quantization.py:
    55-262) as BigCodecDecoder builds it for fsq=True (codec_decoder.py:41-47: levels, channel_first=True,
    dim=in_channels; one codebook, nn.Linear projections with bias; the same state_dict keys
    project_in.weight/bias, project_out.weight/bias).  Eval forward: one bc_fsq_fwd launch,
    z (B, D, T) -> (project_out(codes) (B, D, T), indices (B, T) int32)."""

    def __init__(self, levels, dim=None, num_codebooks=1, channel_first=False, projection_has_bias=True, **_):
        super().__init__()
        if num_codebooks != 1 or not projection_has_bias:
            raise NotImplementedError("FSQ: one codebook with biased projections (the decoder's use)")
        self.levels = [int(v) for v in levels]
        if not 1 <= len(self.levels) <= 8:
            raise NotImplementedError("FSQ: 1..8 levels")
        self.codebook_dim = len(self.levels)
        self.dim = dim if dim is not None else self.codebook_dim
        self.channel_first = channel_first
        self.codebook_size = int(np.prod(self.levels))
        self.has_projections = self.dim != self.codebook_dim
        self.project_in = nn.Linear(self.dim, self.codebook_dim) if self.has_projections else nn.Identity()
        self.project_out = nn.Linear(self.codebook_dim, self.dim) if self.has_projections else nn.Identity()
        self._cache = _DeviceCache()

    def constants(self) -> torch.Tensor:
        """[5][d] float32 = half_l, offset, shift, half_width, basis, from the reference's own torch
        expressions (bound :118-123, quantize :147-149, codes_to_indices :164-168), on the CPU."""
        lv = torch.tensor(self.levels, dtype=torch.int32)
        half_l = (lv - 1) * (1 + 1e-3) / 2
        offset = torch.where(lv % 2 == 0, 0.5, 0.0)
        shift = (offset / half_l).atanh()
        hw = lv // 2
        basis = torch.cumprod(torch.tensor([1] + self.levels[:-1]), dim=0, dtype=torch.int32)
        return torch.stack([half_l.float(), offset.float(), shift.float(), hw.float(), basis.float()]).contiguous()

    def prepared(self, device):
        lin_in, lin_out = self.project_in, self.project_out
        src = [lin_in.weight, lin_in.bias, lin_out.weight, lin_out.bias] if self.has_projections else []

        def build():
            if self.has_projections:
                w_in, b_in, w_out, b_out = (_cpu(t).contiguous() for t in src)
            else:  # identity projections: exact through the fma chains (x * 1 + 0)
                w_in = w_out = torch.eye(self.dim)
                b_in = b_out = torch.zeros(self.dim)
            return tuple(t.to(device) for t in (w_in, b_in, w_out, b_out, self.constants()))
        return self._cache.get(_pkey(*src) + (str(device),), build)

    def forward(self, z):
        if self.training and torch.is_grad_enabled():
            raise NotImplementedError("training-mode FSQ is out of scope of the HIP inference path; call .eval()")
        if not self.channel_first:
            raise NotImplementedError("FSQ on the HIP path takes channel-first (B, D, T) input, as the decoder uses it")
        z = _as_input(z)
        B, D, T = z.shape
        if D != self.dim:
            raise ValueError(f"expected dimension of {self.dim} but found dimension of {D}")
        w_in, b_in, w_out, b_out, consts = self.prepared(z.device)
        post, idx = _ops().fsq(z, w_in, b_in, w_out, b_out, consts)
        return post, idx

    def indices_to_codes(self, indices):
        """finite_scalar_quantization.py:176-192 for the decoder's FSQ (channel_first, one codebook): indices
        (B, T) int32 / int64 on the device -> project_out(codes) (B, D, T), one bc_fsq_codes launch (torch's
        floor // and % included: any integer maps to a grid point, as in the reference)."""
        if indices is None:
            raise AssertionError  # the reference's `assert exists(indices)`
        if not self.channel_first or indices.dim() != 2:
            raise NotImplementedError("FSQ.indices_to_codes on the HIP path takes (B, T) indices, channel_first")
        if indices.device.type != "cuda":
            raise L.BigCodecLibraryError("FSQ.indices_to_codes takes device index tensors")
        w_in, b_in, w_out, b_out, consts = self.prepared(indices.device)
        return _ops().fsq_codes(indices.contiguous(), w_out, b_out, self.levels)
