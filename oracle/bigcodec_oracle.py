"""CPU oracle for the BigCodec tokenization path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / baseline.  The product (audiotokenization_amd) never imports it.

This is a functional restatement, on the torch CPU ops the reference itself runs on (the
reference's arithmetic lives in aten CPU kernels: oneDNN conv, mkldnn LSTM, MKL sgemm, vectorised
sin/exp; torch 2.10.0 in this image), of the reference's forward path, driven by a flat state_dict
with the reference's own key names:

  encoder_forward   vq/codec_encoder.py:35-64
  decoder_forward   vq/codec_decoder.py:59-94 (vq=False path)
  rvq_forward       vq/residual_vq.py:21-40 + vq/factorized_vector_quantize.py:29-76, 93-108
  vq2emb            vq/residual_vq.py:42-48 + vq/factorized_vector_quantize.py:78-91
  fsq_forward       vq/vector_quantize_pytorch_lucidrains/finite_scalar_quantization.py:205-262 (fsq=True)

Pinning: tests/test_oracle_pinned.py checks this restatement bit-for-bit (torch.equal) against the
reference modules imported from /root/reference (in the development container only) and against
the committed golden fixtures in tests/golden/ produced by tools/make_golden.py from the reference.
"""
from __future__ import annotations

from typing import Dict, Mapping, Sequence

import numpy as np
import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Mapping[str, Tensor]


# --------------------------------------------------------------------------------------------
# leaf ops
# --------------------------------------------------------------------------------------------
def wn_weight(sd: SD, prefix: str) -> Tensor:
    """weight_norm (dim 0) as torch.nn.utils.weight_norm recomputes it on every forward
    (vq/module.py:59-72).  A plain `weight` (after remove_weight_norm) is used as is."""
    if prefix + "weight" in sd:
        return sd[prefix + "weight"]
    return torch._weight_norm(sd[prefix + "weight_v"], sd[prefix + "weight_g"], 0)


def snake_beta(x: Tensor, alpha: Tensor, beta: Tensor, logscale: bool = True) -> Tensor:
    """SnakeBeta.forward, vq/activations.py:107-118 (same op order)."""
    alpha = alpha.unsqueeze(0).unsqueeze(-1)
    beta = beta.unsqueeze(0).unsqueeze(-1)
    if logscale:
        alpha = torch.exp(alpha)
        beta = torch.exp(beta)
    return x + (1.0 / (beta + 0.000000001)) * torch.pow(torch.sin(x * alpha), 2)


def upsample2(x: Tensor, filt: Tensor, ratio: int = 2) -> Tensor:
    """UpSample1d(ratio, kernel).forward, vq/alias_free_torch/resample.py:10-33 (default ratio 2, 12 taps)."""
    C = x.shape[1]
    k = filt.shape[-1]
    pad = k // ratio - 1
    pad_left = pad * ratio + (k - ratio) // 2
    pad_right = pad * ratio + (k - ratio + 1) // 2
    x = F.pad(x, (pad, pad), mode="replicate")
    x = ratio * F.conv_transpose1d(x, filt.expand(C, -1, -1), stride=ratio, groups=C)
    return x[..., pad_left:-pad_right]


def downsample2(x: Tensor, filt: Tensor, ratio: int = 2) -> Tensor:
    """DownSample1d(ratio, kernel) -> LowPassFilter1d.forward, resample.py:36-49, filter.py:86-95."""
    C = x.shape[1]
    k = filt.shape[-1]
    even = k % 2 == 0
    pad_left = k // 2 - int(even)
    pad_right = k // 2
    x = F.pad(x, (pad_left, pad_right), mode="replicate")
    return F.conv1d(x, filt.expand(C, -1, -1), stride=ratio, groups=C)


def activation(x: Tensor, sd: SD, prefix: str, antialias: bool, up_ratio: int = 2, down_ratio: int = 2) -> Tensor:
    """Activation1d(SnakeBeta).forward, vq/alias_free_torch/act.py:25-32."""
    if antialias:
        x = upsample2(x, sd[prefix + "upsample.filter"], up_ratio)
    x = snake_beta(x, sd[prefix + "act.alpha"], sd[prefix + "act.beta"])
    if antialias:
        x = downsample2(x, sd[prefix + "downsample.lowpass.filter"], down_ratio)
    return x


def conv(x: Tensor, sd: SD, prefix: str, kernel_size: int, stride: int = 1, padding: int = 0,
         dilation: int = 1, causal: bool = False) -> Tensor:
    """WNConv1d / CausalConv1d forward, vq/module.py:45-48, 59-65."""
    if causal:
        p = prefix + "conv."
        w = wn_weight(sd, p)
        x = F.pad(x, ((kernel_size - stride) * dilation, 0), mode="constant")
        return F.conv1d(x, w, sd.get(p + "bias"), stride, 0, dilation)
    w = wn_weight(sd, prefix)
    return F.conv1d(x, w, sd.get(prefix + "bias"), stride, padding, dilation)


def conv_transpose(x: Tensor, sd: SD, prefix: str, stride: int, causal: bool) -> Tensor:
    """WNConvTranspose1d / CausalConvTranspose1d forward, vq/module.py:50-57, 67-72, with the
    DecoderBlock's padding / output_padding (vq/module.py:118-124)."""
    if causal:
        p = prefix + "conv."
        w = wn_weight(sd, p)
        return F.conv_transpose1d(x, w, sd.get(p + "bias"), stride)[..., :-stride]
    pad = stride // 2 + stride % 2 if stride != 1 else 0
    opad = stride % 2 if stride != 1 else 0
    w = wn_weight(sd, prefix)
    return F.conv_transpose1d(x, w, sd.get(prefix + "bias"), stride, pad, opad)


# --------------------------------------------------------------------------------------------
# blocks
# --------------------------------------------------------------------------------------------
def residual_unit(x: Tensor, sd: SD, prefix: str, dilation: int, causal: bool, antialias: bool) -> Tensor:
    """ResidualUnit.forward, vq/module.py:74-89."""
    pad = 0 if causal else ((7 - 1) * dilation) // 2
    y = activation(x, sd, prefix + "block.0.", antialias)
    y = conv(y, sd, prefix + "block.1.", 7, 1, pad, dilation, causal)
    y = activation(y, sd, prefix + "block.2.", antialias)
    y = conv(y, sd, prefix + "block.3.", 1)
    return x + y


def encoder_block(x: Tensor, sd: SD, prefix: str, stride: int, dilations: Sequence[int], causal: bool,
                  antialias: bool) -> Tensor:
    """EncoderBlock.forward, vq/module.py:91-113."""
    for i, d in enumerate(dilations):
        x = residual_unit(x, sd, f"{prefix}block.{i}.", d, causal, antialias)
    n = len(dilations)
    x = activation(x, sd, f"{prefix}block.{n}.", antialias)
    pad = 0 if causal else (stride // 2 + stride % 2 if stride != 1 else 0)
    k = 2 * stride if stride != 1 else 1
    return conv(x, sd, f"{prefix}block.{n + 1}.", k, stride, pad, 1, causal)


def decoder_block(x: Tensor, sd: SD, prefix: str, stride: int, dilations: Sequence[int], causal: bool,
                  antialias: bool) -> Tensor:
    """DecoderBlock.forward, vq/module.py:115-141."""
    x = activation(x, sd, f"{prefix}block.0.", antialias)
    x = conv_transpose(x, sd, f"{prefix}block.1.", stride, causal)
    for i, d in enumerate(dilations):
        x = residual_unit(x, sd, f"{prefix}block.{i + 2}.", d, causal, antialias)
    return x


def res_lstm(x: Tensor, sd: SD, prefix: str, num_layers: int, bidirectional: bool = False) -> Tensor:
    """ResLSTM.forward, vq/module.py:156-167, on torch's own CPU LSTM (the reference's arithmetic)."""
    dim = x.shape[1]
    lstm = torch.nn.LSTM(dim, dim if not bidirectional else dim // 2, num_layers, batch_first=True,
                         bidirectional=bidirectional)
    lstm.load_state_dict({k[len(prefix) + 5:]: v for k, v in sd.items() if k.startswith(prefix + "lstm.")})
    xt = x.transpose(1, 2)
    with torch.no_grad():
        y, _ = lstm(xt)
    y = y + xt
    return y.transpose(1, 2)


# --------------------------------------------------------------------------------------------
# models
# --------------------------------------------------------------------------------------------
def encoder_forward(x: Tensor, sd: SD, cfg: Mapping) -> Tensor:
    """BigCodecEncoder.forward (vq/codec_encoder.py:35-64).  x (B,1,T) -> (B, D, T/hop)."""
    causal, aa = cfg.get("causal", False), cfg.get("antialias", False)
    dil = tuple(cfg.get("dilations", (1, 3, 9)))
    i = 0
    x = conv(x, sd, f"block.{i}.", 7, 1, 3, 1, causal)
    for stride in cfg["up_ratios"]:
        i += 1
        x = encoder_block(x, sd, f"block.{i}.", stride, dil, causal, aa)
    if cfg.get("use_rnn", True):
        i += 1
        x = res_lstm(x, sd, f"block.{i}.", cfg.get("rnn_num_layers", 2), cfg.get("rnn_bidirectional", False))
    i += 1
    x = activation(x, sd, f"block.{i}.", aa)
    i += 1
    return conv(x, sd, f"block.{i}.", 3, 1, 1, 1, causal)


def decoder_forward(x: Tensor, sd: SD, cfg: Mapping) -> Tensor:
    """BigCodecDecoder.forward(x, vq=False) (vq/codec_decoder.py:59-94).  (B,D,F) -> (B,1,T)."""
    causal, aa = cfg.get("causal", False), cfg.get("antialias", False)
    dil = tuple(cfg.get("dilations", (1, 3, 9)))
    i = 0
    x = conv(x, sd, f"model.{i}.", 7, 1, 3, 1, causal)
    if cfg.get("use_rnn", True):
        i += 1
        x = res_lstm(x, sd, f"model.{i}.", cfg.get("rnn_num_layers", 2), cfg.get("rnn_bidirectional", False))
    for stride in cfg["up_ratios"]:
        i += 1
        x = decoder_block(x, sd, f"model.{i}.", stride, dil, causal, aa)
    i += 1
    x = activation(x, sd, f"model.{i}.", aa)
    i += 1
    x = conv(x, sd, f"model.{i}.", 7, 1, 3, 1, causal)
    return torch.tanh(x)


def _linear(x: Tensor, sd: SD, prefix: str) -> Tensor:
    return F.linear(x, wn_weight(sd, prefix), sd[prefix + "bias"])


def decode_latents(latents: Tensor, codebook: Tensor):
    """FactorizedVectorQuantize.decode_latents, vq/factorized_vector_quantize.py:93-108."""
    b = latents.size(0)
    enc = latents.permute(0, 2, 1).reshape(-1, latents.shape[1])
    enc = F.normalize(enc)
    cb = F.normalize(codebook)
    dist = enc.pow(2).sum(1, keepdim=True) - 2 * enc @ cb.t() + cb.pow(2).sum(1, keepdim=True).t()
    indices = (-dist).max(1)[1].reshape(b, -1)
    z_q = F.embedding(indices, codebook).transpose(1, 2)
    return z_q, indices


def fvq_forward(z: Tensor, sd: SD, prefix: str, return_ze: bool = False):
    """FactorizedVectorQuantize.forward (eval), vq/factorized_vector_quantize.py:29-76."""
    zt = z.permute(0, 2, 1)
    has_proj = (prefix + "in_proj.weight_v") in sd or (prefix + "in_proj.weight") in sd
    z_e = _linear(zt, sd, prefix + "in_proj.") if has_proj else zt
    z_e = z_e.permute(0, 2, 1)
    z_q, indices = decode_latents(z_e, sd[prefix + "_codebook.weight"])
    commit_loss = torch.zeros(z.shape[0])
    z_q = z_e + (z_q - z_e).detach()
    z_q = z_q.permute(0, 2, 1)
    if has_proj:
        z_q = _linear(z_q, sd, prefix + "out_proj.")
    z_q = z_q.permute(0, 2, 1)
    if return_ze:
        return z_q, indices, commit_loss, z_e
    return z_q, indices, commit_loss


def rvq_forward(x: Tensor, sd: SD, prefix: str = "quantizer.", num_quantizers: int = 1):
    """ResidualVQ.forward, vq/residual_vq.py:21-40 -> (quantized (B,D,F), indices (Nq,B,F), losses (Nq,))."""
    quantized_out = 0.0
    residual = x
    losses, indices = [], []
    for q in range(num_quantizers):
        quantized, idx, loss = fvq_forward(residual, sd, f"{prefix}layers.{q}.")
        residual = residual - quantized
        quantized_out = quantized_out + quantized
        losses.append(loss.mean())
        indices.append(idx)
    return quantized_out, torch.stack(indices), torch.stack(losses)


def vq2emb(vq: Tensor, sd: SD, prefix: str = "quantizer.", num_quantizers: int = 1, proj: bool = True) -> Tensor:
    """ResidualVQ.vq2emb (vq/residual_vq.py:42-48): vq (B,T,Nq) -> (B,T,D)."""
    out = 0.0
    for q in range(num_quantizers):
        p = f"{prefix}layers.{q}."
        emb = F.embedding(vq[:, :, q], sd[p + "_codebook.weight"])
        if proj and ((p + "out_proj.weight_v") in sd or (p + "out_proj.weight") in sd):
            emb = _linear(emb, sd, p + "out_proj.")
        out = out + emb
    return out


def fsq_forward(z: Tensor, sd: SD, levels: Sequence[int], prefix: str = "quantizer."):
    """FSQ.forward (vq/vector_quantize_pytorch_lucidrains/finite_scalar_quantization.py:205-262) as the
    fsq=True decoder calls it (codec_decoder.py:41-47, 87-88): eval, channel_first, one codebook,
    projections with bias.  z (B, D, T) -> (out (B, D, T), indices (B, T) int32)."""
    lv = torch.tensor(list(levels), dtype=torch.int32)
    basis = torch.cumprod(torch.tensor([1] + list(levels[:-1])), dim=0, dtype=torch.int32)
    x = z.transpose(1, 2)  # rearrange b d ... -> b ... d (pack_one is a no-op for 3-D input)
    if (prefix + "project_in.weight") in sd:
        x = F.linear(x, sd[prefix + "project_in.weight"], sd[prefix + "project_in.bias"])
    x = x[:, :, None, :]  # b n (c d) -> b n c d, c = 1
    half_l = (lv - 1) * (1 + 1e-3) / 2  # bound (:118-123)
    offset = torch.where(lv % 2 == 0, 0.5, 0.0)
    shift = (offset / half_l).atanh()
    bounded = (x + shift).tanh() * half_l - offset
    quantized = bounded + (bounded.round() - bounded)  # round_ste forward value (:49-52)
    half_width = lv // 2
    codes = quantized / half_width  # quantize (:147-149)
    indices = ((codes * half_width + half_width) * basis).sum(dim=-1).to(torch.int32)  # codes_to_indices
    codes = codes.reshape(codes.shape[0], codes.shape[1], -1)
    if (prefix + "project_out.weight") in sd:
        codes = F.linear(codes, sd[prefix + "project_out.weight"], sd[prefix + "project_out.bias"])
    return codes.transpose(1, 2), indices[..., 0]


def fsq_indices_to_codes(indices: Tensor, sd: SD, levels: Sequence[int], prefix: str = "quantizer."):
    """FSQ.indices_to_codes (finite_scalar_quantization.py:159-192) for the fsq=True decoder's quantizer
    (channel_first, one codebook): indices (B, T) integer -> project_out(codes) (B, D, T).  Level indices by
    torch's floor // and % (:170-174), so any integer lands on the grid."""
    lv = torch.tensor(list(levels), dtype=torch.int32)
    basis = torch.cumprod(torch.tensor([1] + list(levels[:-1])), dim=0, dtype=torch.int32)
    level_idx = (indices[..., None] // basis) % lv
    half_width = lv // 2
    codes = (level_idx - half_width) / half_width  # _scale_and_shift_inverse (:155-157)
    if (prefix + "project_out.weight") in sd:
        codes = F.linear(codes, sd[prefix + "project_out.weight"], sd[prefix + "project_out.bias"])
    return codes.transpose(1, 2)


def strip_prefix(sd: Mapping[str, Tensor], prefix: str) -> Dict[str, Tensor]:
    return {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}


def to_torch_sd(sd_np: Mapping[str, np.ndarray]) -> Dict[str, Tensor]:
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd_np.items()}


@torch.no_grad()
def encode_indices(wav: Tensor, enc_sd: SD, dec_sd: SD, enc_cfg: Mapping, dec_cfg: Mapping):
    """extract_indices.py:353-355 intended path: encoder -> decoder(vq=True) -> codes (Nq,B,F)."""
    emb = encoder_forward(wav, enc_sd, enc_cfg)
    _, codes, _ = rvq_forward(emb, dec_sd, "quantizer.", dec_cfg.get("vq_num_quantizers", 1))
    return codes, emb
