"""Generate tests/golden/fsq_*.npz from the REFERENCE decoder with fsq=True (codec_decoder.py:41-47, 85-92;
the vendored lucidrains FSQ, vq/vector_quantize_pytorch_lucidrains/finite_scalar_quantization.py).

Run in the development container only (the reference never travels):
    python tools/make_golden_fsq.py
Fixture = data: the latents fed to the quantizer (the reference debug / base encoder's output on synthetic
clips, scaled to exercise every level), the reference's quantized output, its indices, the fp64 distance
of every bounded coordinate to its nearest rounding boundary (the certificate for an index flip), the
decoded waveform, and the FSQ's indices_to_codes of its own indices and of out-of-range / negative integers.  Weights are not stored: both sides synthesise them (synth.synth_state_dict).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)

import refimport  # noqa: E402
from make_golden import build_ref  # noqa: E402
from audiotokenization_amd import synth  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")


@torch.no_grad()
def fsq_case(ref, name, n_clips, n_samples, levels, gain, random_frames=0):
    cb = int(np.prod(levels))
    enc, dec, ek, dk = build_ref(ref, name, fsq=True, fsq_levels=list(levels), codebook_size=cb)
    if random_frames:  # N(0, gain^2) latents: project_in's output covers most of the level grid
        g = torch.Generator().manual_seed(5)
        z = torch.randn(n_clips, enc.enc_dim if hasattr(enc, "enc_dim") else dk["in_channels"], random_frames,
                        generator=g) * gain
    else:
        x = torch.from_numpy(synth.synth_clips(n_clips, n_samples, clip0=7)).unsqueeze(1)
        z = enc(x) * gain  # spread project_in's output over the levels
    post, q, loss = dec(z, vq=True)
    fsq = dec.quantizer
    zi = fsq.project_in(z.transpose(1, 2)).double()  # (B, F, d) in fp64 for the certificate
    lv = torch.tensor(levels, dtype=torch.float64)
    half_l = (lv - 1) * (1 + 1e-3) / 2
    offset = torch.where(lv % 2 == 0, 0.5, 0.0).double()
    shift = (offset / half_l).atanh()
    bounded = (zi + shift).tanh() * half_l - offset
    margin = ((bounded - bounded.floor()) - 0.5).abs().amin(dim=-1)  # distance to the nearest .5 boundary
    wav = dec(post, vq=False)
    # token -> latent (finite_scalar_quantization.py:176-192; the decoder's own vq2emb has no FSQ branch):
    # the reference's indices_to_codes of its own indices, and of integers outside [0, codebook_size) and
    # negative ones (torch's floor // and % wrap them onto the grid)
    tok_post = fsq.indices_to_codes(q)
    g = torch.Generator().manual_seed(11)
    wrap_idx = torch.cat([torch.randint(-3 * cb, 4 * cb, (q.shape[0], 29), generator=g),
                          torch.tensor([[-1, cb, cb - 1, -cb, 2 * cb + 1, 0, -(cb + 1)]] * q.shape[0])], dim=1)
    wrap_post = fsq.indices_to_codes(wrap_idx)
    out = dict(z=z.numpy(), post=post.numpy(), codes=q.numpy().astype(np.int32), margin=margin.float().numpy(),
               wav=wav.numpy(), loss=loss.numpy(), tok_post=tok_post.numpy(), wrap_idx=wrap_idx.numpy(),
               wrap_post=wrap_post.numpy())
    meta = dict(model=name, overrides=dict(fsq=True, fsq_levels=list(levels), codebook_size=cb), gain=gain,
                torch=torch.__version__, levels=list(levels))
    tag = f"fsq_{name}_" + "x".join(map(str, levels)) + ("_rand" if random_frames else "")
    np.savez_compressed(os.path.join(OUT, tag + ".npz"), meta=json.dumps(meta), **out)
    used = len(np.unique(out["codes"]))
    print(f"{tag}: z {tuple(z.shape)} codes {tuple(q.shape)} {used} distinct of {cb}, min margin {margin.min():.2e}")


def main():
    ref = refimport.load()
    torch.manual_seed(0)
    fsq_case(ref, "debug", 2, 12000, (4, 4, 4, 8), gain=4.0)
    fsq_case(ref, "base", 1, 9600, (8, 5, 5, 5), gain=4.0)
    fsq_case(ref, "debug", 2, 0, (4, 4, 4, 8), gain=3.0, random_frames=64)


if __name__ == "__main__":
    main()
