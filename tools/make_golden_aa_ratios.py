"""Generate tests/golden/aa_activation_ratios.npz from the REFERENCE's Activation1d with non-default
constructor arguments (vq/alias_free_torch/act.py:8-23: up_ratio, down_ratio, up/down kernel sizes; no
shipped config sets them).  Development container only (the reference never travels):
    python tools/make_golden_aa_ratios.py
Data only: random inputs / Snake parameters and the reference's outputs and filter buffers.
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

import refimport  # noqa: E402

# (up_ratio, down_ratio, up_kernel_size, down_kernel_size); None = the reference's default int(6 r / 2) * 2
CASES = [(3, 3, None, None), (2, 2, 8, 10), (4, 2, None, None), (2, 4, None, None), (2, 2, 12, 11), (1, 1, 6, 5)]


@torch.no_grad()
def main():
    ref = refimport.load()
    g = torch.Generator().manual_seed(1234)
    out = {}
    for ci, (ru, rd, ku, kd) in enumerate(CASES):
        for T in (1, 7, 300):
            act = ref.alias_free.Activation1d(activation=ref.activations.SnakeBeta(5, alpha_logscale=True),
                                              antialias=True, up_ratio=ru, down_ratio=rd,
                                              up_kernel_size=ku, down_kernel_size=kd)
            act.act.alpha.copy_(torch.rand(5, generator=g) - 0.5)
            act.act.beta.copy_(torch.rand(5, generator=g) - 0.5)
            x = torch.randn(2, 5, T, generator=g)
            k = f"c{ci}_T{T}"
            out[f"x_{k}"] = x.numpy()
            out[f"alpha_{k}"] = act.act.alpha.numpy()
            out[f"beta_{k}"] = act.act.beta.numpy()
            out[f"y_{k}"] = act(x).numpy()
        out[f"up_filter_c{ci}"] = act.upsample.filter.numpy()
        out[f"down_filter_c{ci}"] = act.downsample.lowpass.filter.numpy()
    meta = dict(torch=torch.__version__, cases=CASES, T=[1, 7, 300])
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "aa_activation_ratios.npz"), meta=json.dumps(meta), **out)
    print("aa_activation_ratios", len(CASES))


if __name__ == "__main__":
    main()
