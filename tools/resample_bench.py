"""Time the GPU sinc resampler (bc_resample_sinc) on a batch of clips, as the ingest path runs it.

    python tools/resample_bench.py [--B 64] [--seconds 10] [--orig 16000] [--new 24000] [--iters 20]

Prints ms per launch and the algorithmic HBM rate (4 B read per input sample + 4 B written per output
sample) against the 8 TB/s HBM3E peak.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from audiotokenization_amd import ingest  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--B", type=int, default=64)
    p.add_argument("--seconds", type=float, default=10.0)
    p.add_argument("--orig", type=int, default=16000)
    p.add_argument("--new", type=int, default=24000)
    p.add_argument("--iters", type=int, default=20)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    n = int(a.seconds * a.orig)
    x = torch.randn(a.B, n, device=dev)
    rs = ingest.Resampler.get(a.orig, a.new, dev)
    y = rs(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        y = rs(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    nbytes = 4.0 * (x.numel() + y.numel())
    gbs = nbytes / ms / 1e6
    print(f"resample {a.orig}->{a.new} B={a.B} {a.seconds:g} s: {ms:.3f} ms/launch, {nbytes / 1e9:.3f} GB, "
          f"{gbs:.0f} GB/s = {gbs / 8000:.3f} of 8 TB/s; {a.B * a.seconds / (ms * 1e-3):.0f} audio-s/s; "
          f"{rs.new} phases x {rs.taps} taps", flush=True)


if __name__ == "__main__":
    main()
