"""Full-size fixtures from the REFERENCE modules (SURVEY §8(c) "Golden vectors to commit" items 2-3),
plus the LSTM-length and multi-quantizer pins VERDICT r01 asked for.

Run in the development container only (the reference never travels; tools/refimport.py):
    python tools/make_golden_full.py [config2] [config3] [long30] [rvq]

* config2  -> tests/golden/full_config2_default.npz: 64 x 240 000-sample clips (synth.synth_clips,
             clips 0..63 = bench.py's rank-0 batch), `default` model, reference encode + VQ run B = 1 per
             clip as extract_indices.py:397/510 does; int16 indices (64, 1200), the fp64 top-2 distance
             gap of every frame, the full latent of clip 0 and 16 fp64 random-projection fingerprints
             of every clip's latent.
* config3  -> tests/golden/full_config3_default.npz: the same clips through the reference decoder
             (vq=False on the reference's own post-VQ embedding, inference_full.py:557-561): waveforms
             of clips 0-1, and per clip sum(y^2), sum(y) and 16 fp64 random-projection fingerprints.
* long30   -> tests/golden/long30_default.npz: one 720 000-sample (30 s) clip (T = 3600 LSTM steps, the
             config-5 length): indices, gaps, latent fingerprints and the latent's last 64 frames.
* rvq      -> tests/golden/rvq_base_nq{2,4}.npz: `base` model with vq_num_quantizers = 2 / 4
             (residual_vq.py:21-40): codes (Nq, B, F), the per-layer fp64 gap of every frame (the residual
             each layer sees), post-VQ embedding, losses, and vq2emb.

Fingerprint projections are generated from a fixed numpy seed (PROJ_SEED) so tests rebuild them.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import refimport  # noqa: E402
from make_golden import build_ref, top2_gap  # noqa: E402
from audiotokenization_amd import synth  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
PROJ_SEED = 20261016
N_PROJ = 16


def projections(shape, n=N_PROJ, seed=PROJ_SEED):
    """(n, *shape) float64 +-1 projection vectors (tests regenerate them with the same call)."""
    rng = np.random.default_rng(seed)
    return rng.integers(0, 2, size=(n,) + tuple(shape)).astype(np.float64) * 2.0 - 1.0


def fingerprint(a: np.ndarray, proj: np.ndarray) -> np.ndarray:
    """16 fp64 dot products of one clip's array with the projection vectors."""
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    return proj.reshape(proj.shape[0], -1) @ a


@torch.no_grad()
def config2(ref, n_clips=64, n_samples=240_000):
    t0 = time.time()
    enc, dec, ek, dk = build_ref(ref, "default")
    fvq = dec.quantizer.layers[0]
    codes = np.zeros((n_clips, n_samples // 200), np.int16)
    gaps = np.zeros((n_clips, n_samples // 200), np.float32)
    lat_fp = np.zeros((n_clips, N_PROJ), np.float64)
    proj = None
    lat0 = None
    posts = []
    for i in range(n_clips):
        x = torch.from_numpy(synth.synth_clips(1, n_samples, clip0=i)).unsqueeze(1)
        emb = enc(x)                                       # extract_indices.py:510 -> BigCodecEncoder
        post, c, _ = dec(emb, vq=True)                     # codes (1, 1, F)
        z_e = fvq.in_proj(emb.transpose(1, 2)).transpose(1, 2)
        codes[i] = c[0, 0].numpy().astype(np.int16)        # extract_indices.py:520-532
        gaps[i] = top2_gap(z_e, fvq.codebook.weight)[0]
        if proj is None:
            proj = projections(emb.shape[1:])
        lat_fp[i] = fingerprint(emb[0].numpy(), proj)
        if i == 0:
            lat0 = emb[0].numpy()
        posts.append(post)
        print(f"config2 clip {i}: {time.time() - t0:.0f} s, min gap {gaps[i].min():.2e}", flush=True)
    meta = dict(model="default", n_clips=n_clips, n_samples=n_samples, torch=torch.__version__, proj_seed=PROJ_SEED,
                n_proj=N_PROJ, batch=1, seconds=round(time.time() - t0, 1), encoder_kwargs=ek, decoder_kwargs=dk)
    np.savez_compressed(os.path.join(OUT, "full_config2_default.npz"), meta=json.dumps(meta), codes=codes, gap=gaps,
                        latent0=lat0, latent_fp=lat_fp)
    print("full_config2_default", meta["seconds"], "s", flush=True)
    return dec, posts


@torch.no_grad()
def config3(ref, dec=None, posts=None, n_clips=64, n_samples=240_000):
    t0 = time.time()
    if dec is None:
        enc, dec, ek, dk = build_ref(ref, "default")
        posts = []
        for i in range(n_clips):
            x = torch.from_numpy(synth.synth_clips(1, n_samples, clip0=i)).unsqueeze(1)
            posts.append(dec(enc(x), vq=True)[0])
    proj = projections((n_samples,))
    sumsq = np.zeros(n_clips, np.float64)
    sums = np.zeros(n_clips, np.float64)
    wfp = np.zeros((n_clips, N_PROJ), np.float64)
    wav01 = []
    for i in range(n_clips):
        y = dec(posts[i], vq=False)[0, 0].numpy()          # inference_full.py:561
        yd = y.astype(np.float64)
        sumsq[i] = float((yd * yd).sum())
        sums[i] = float(yd.sum())
        wfp[i] = fingerprint(yd, proj)
        if i < 2:
            wav01.append(y)
        print(f"config3 clip {i}: {time.time() - t0:.0f} s", flush=True)
    meta = dict(model="default", n_clips=n_clips, n_samples=n_samples, torch=torch.__version__, proj_seed=PROJ_SEED,
                n_proj=N_PROJ, batch=1, seconds=round(time.time() - t0, 1))
    np.savez_compressed(os.path.join(OUT, "full_config3_default.npz"), meta=json.dumps(meta), wav01=np.stack(wav01),
                        sumsq=sumsq, sum=sums, wav_fp=wfp)
    print("full_config3_default", meta["seconds"], "s", flush=True)


@torch.no_grad()
def long30(ref, n_samples=720_000, clip=0):
    t0 = time.time()
    enc, dec, ek, dk = build_ref(ref, "default")
    fvq = dec.quantizer.layers[0]
    x = torch.from_numpy(synth.synth_clips(1, n_samples, clip0=clip)).unsqueeze(1)
    emb = enc(x)
    post, c, _ = dec(emb, vq=True)
    z_e = fvq.in_proj(emb.transpose(1, 2)).transpose(1, 2)
    proj = projections(emb.shape[1:])
    meta = dict(model="default", n_clips=1, clip0=clip, n_samples=n_samples, torch=torch.__version__,
                proj_seed=PROJ_SEED, n_proj=N_PROJ, seconds=round(time.time() - t0, 1))
    np.savez_compressed(os.path.join(OUT, "long30_default.npz"), meta=json.dumps(meta),
                        codes=c[0, 0].numpy().astype(np.int16), gap=top2_gap(z_e, fvq.codebook.weight)[0],
                        latent_fp=fingerprint(emb[0].numpy(), proj), latent_tail=emb[0, :, -64:].numpy())
    print("long30_default", meta["seconds"], "s", flush=True)


@torch.no_grad()
def rvq(ref, nq, n_clips=2, n_samples=24_000):
    """ResidualVQ with nq layers (residual_vq.py:21-40) on the base model's encoder latent."""
    enc, dec, ek, dk = build_ref(ref, "base", vq_num_quantizers=nq)
    x = torch.from_numpy(synth.synth_clips(n_clips, n_samples, clip0=3)).unsqueeze(1)
    lat = enc(x)
    post, codes, losses = dec(lat, vq=True)
    # per-layer gaps on the residual each layer sees (same loop as residual_vq.py:28-36)
    gaps = []
    residual = lat
    for layer in dec.quantizer.layers:
        z_e = layer.in_proj(residual.transpose(1, 2)).transpose(1, 2)
        gaps.append(top2_gap(z_e, layer.codebook.weight))
        q, _, _ = layer(residual)
        residual = residual - q
    emb2 = dec.vq2emb(codes.permute(1, 2, 0))
    meta = dict(model="base", vq_num_quantizers=nq, n_clips=n_clips, n_samples=n_samples, clip0=3,
                torch=torch.__version__, encoder_kwargs=ek, decoder_kwargs=dk)
    np.savez_compressed(os.path.join(OUT, f"rvq_base_nq{nq}.npz"), meta=json.dumps(meta), latent=lat.numpy(),
                        codes=codes.numpy(), gap=np.stack(gaps), post=post.numpy(), losses=losses.numpy(),
                        vq2emb=emb2.numpy())
    print(f"rvq_base_nq{nq}", codes.shape, flush=True)


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(int(os.environ.get("GOLDEN_THREADS", "8")))
    ref = refimport.load()
    what = sys.argv[1:] or ["rvq", "long30", "config2", "config3"]
    if "rvq" in what:
        rvq(ref, 2)
        rvq(ref, 4)
    if "long30" in what:
        long30(ref)
    dec = posts = None
    if "config2" in what:
        dec, posts = config2(ref)
    if "config3" in what:
        config3(ref, dec, posts)


if __name__ == "__main__":
    main()
