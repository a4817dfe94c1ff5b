"""Shared test helpers: build models with the synthetic weight spec, oracle state dicts, tolerances."""
from __future__ import annotations

import numpy as np
import torch

from audiotokenization_amd import config as cfgmod
from audiotokenization_amd import synth
from audiotokenization_amd.codec import BigCodecDecoder, BigCodecEncoder


def synth_load(module: torch.nn.Module, prefix: str, seed: int = 0) -> dict:
    """Load the synthetic spec into `module` (keys prefixed like the Lightning module) and return
    the module-level numpy state dict."""
    sd = module.state_dict()
    full = {prefix + k: v for k, v in sd.items()}
    syn = synth.synth_state_dict(full, seed=seed)
    local = {k[len(prefix):]: v for k, v in syn.items()}
    module.load_state_dict({k: torch.from_numpy(v) for k, v in local.items()}, strict=True)
    return local


def build_models(name: str, device=None, **ov):
    """(encoder, decoder, enc_sd, dec_sd, enc_cfg, dec_cfg) with synthetic weights."""
    cfg = cfgmod.preset(name, **ov)
    ek = cfgmod.encoder_kwargs(cfg.model.codec_encoder)
    dk = cfgmod.decoder_kwargs(cfg.model.codec_decoder)
    enc = BigCodecEncoder(**ek)
    dec = BigCodecDecoder(**dk)
    esd = synth_load(enc, "encoder.")
    dsd = synth_load(dec, "decoder.")
    enc.eval()
    dec.eval()
    if device is not None:
        enc.to(device)
        dec.to(device)
    return enc, dec, esd, dsd, ek, dk


def torch_sd(sd_np):
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd_np.items()}


def max_rel_err(a, b) -> float:
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    scale = b.abs().max().clamp_min(1e-30)
    return float((a - b).abs().max() / scale)


def error_profile(a, b, top: int = 8) -> str:
    """Where a (C, F) or (..., C, F) difference lives: the frames and channels with the largest |a - b|, the
    error by frame decile and how many elements exceed 10x the median error -- so a failure in a race-free
    kernel path (whole-tensor drift) reads differently from one bad lane / tile / time step."""
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    d = (a - b).abs().reshape(-1, a.shape[-2], a.shape[-1]).amax(0)  # (C, F)
    by_f, by_c = d.amax(0), d.amax(1)
    F = by_f.numel()
    fi = torch.argsort(by_f, descending=True)[:top].tolist()
    ci = torch.argsort(by_c, descending=True)[:top].tolist()
    dec = [float(by_f[i * F // 10:(i + 1) * F // 10].max()) for i in range(10) if (i + 1) * F // 10 > i * F // 10]
    med = float(d.median())
    return ("worst frames " + ", ".join(f"{i}:{float(by_f[i]):.1e}(ch {int(d[:, i].argmax())})" for i in fi) +
            "; worst channels " + ", ".join(f"{i}:{float(by_c[i]):.1e}" for i in ci) +
            "; max by frame decile " + " ".join(f"{v:.1e}" for v in dec) +
            f"; median {med:.1e}, {int((d > 10 * med).sum())} of {d.numel()} above 10x median")


def assert_close_rel(a, b, tol: float, what: str = "", profile: bool = False):
    err = max_rel_err(a, b)
    if err > tol and profile:
        raise AssertionError(f"{what}: max |a-b| / max|b| = {err:.3e} > {tol:.1e}; {error_profile(a, b)}")
    assert err <= tol, f"{what}: max |a-b| / max|b| = {err:.3e} > {tol:.1e}"


def top2_gap(z_e: torch.Tensor, codebook: torch.Tensor) -> np.ndarray:
    """fp64 gap between the best and the second-best VQ distance of every frame of z_e (B, 8, F)."""
    b, d, t = z_e.shape
    e = z_e.permute(0, 2, 1).reshape(-1, d).double()
    e = e / e.norm(dim=1, keepdim=True).clamp_min(1e-12)
    c = codebook.double()
    c = c / c.norm(dim=1, keepdim=True).clamp_min(1e-12)
    dist = (e * e).sum(1, keepdim=True) - 2 * e @ c.t() + (c * c).sum(1)[None]
    v, _ = torch.topk(dist, 2, dim=1, largest=False)
    return (v[:, 1] - v[:, 0]).reshape(b, t).float().numpy()


GAP_TOL = 1e-6  # certified near-tie: an fp32 reassociation can flip a frame only below this gap


def index_mismatches(got, want, gap, gap_tol: float = GAP_TOL, max_frac: float = 1e-3):
    """Compare indices; every mismatch must sit at a frame whose fp64 top-2 distance gap is below
    gap_tol (a near-tie that legitimately flips under fp32 reassociation; SURVEY §0 item 7 measured
    one between two valid CPU builds at 1.2e-7), and at most max_frac of the frames (+1) may differ.
    Returns (n_mismatch, max gap among mismatches)."""
    got = np.asarray(got).reshape(-1)
    want = np.asarray(want).reshape(-1)
    gap = np.asarray(gap).reshape(-1)
    assert got.shape == want.shape == gap.shape, (got.shape, want.shape, gap.shape)
    bad = np.nonzero(got != want)[0]
    worst = float(gap[bad].max()) if bad.size else 0.0
    detail = ", ".join(f"frame {i}: {got[i]} vs {want[i]} (gap {gap[i]:.2e})" for i in bad[:8])
    assert worst <= gap_tol, f"{bad.size} index mismatches, one at a certified gap {worst:.3e} > {gap_tol:.1e}: {detail}"
    assert bad.size <= max_frac * got.size + 1, f"{bad.size} / {got.size} index mismatches: {detail}"
    return bad.size, worst
