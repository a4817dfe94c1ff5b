"""Time the one-launch ResidualUnit (bc_resunit_fwd) at a BigCodec encoder shape.

    python tools/ru_bench.py --C 96 --d 3 --T 120000 [--B 64] [--dual] [--iters 5] [--cfg N]

Prints ms per launch, fp32-equivalent TFLOP/s (k7 + k1) and the algorithmic HBM GB/s
(x_raw + x_act + y [+ y2])."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# BIGCODEC_PKG_ROOT: import the package from another tree (an ablation build under gpurun_abl/)
sys.path.insert(0, os.environ.get("BIGCODEC_PKG_ROOT", REPO))

import torch  # noqa: E402

from audiotokenization_amd import _lib as L  # noqa: E402
from audiotokenization_amd import blocks as BL  # noqa: E402
from audiotokenization_amd.modules import Activation1d, SnakeBeta  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--C", type=int, required=True)
    p.add_argument("--d", type=int, default=1)
    p.add_argument("--T", type=int, default=120000)
    p.add_argument("--B", type=int, default=64)
    p.add_argument("--dual", action="store_true")
    p.add_argument("--iters", type=int, default=5)
    p.add_argument("--cfg", type=int, default=-1)
    p.add_argument("--precision", default="h3")
    p.add_argument("--lazy", action="store_true", help="snake on load (x_act = None), as the encoder flow runs it")
    a = p.parse_args()
    L.set_precision(a.precision)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ru = BL.ResidualUnit(a.C, a.d)
    with torch.no_grad():
        for n, prm in ru.named_parameters():
            prm.copy_(torch.randn_like(prm) * (0.1 if "bias" in n or "alpha" in n or "beta" in n else 1.0))
    nxt = Activation1d(activation=SnakeBeta(a.C, alpha_logscale=True))
    x_raw = torch.randn(a.B, a.C, a.T, device=dev)
    x_act = torch.randn(a.B, a.C, a.T, device=dev)
    cfg = a.cfg if a.cfg >= 0 else ru._fused_cfg()

    def run():
        return ru._flow_fused(cfg, x_raw, None if a.lazy else x_act, a.dual, nxt)

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    fl = 2.0 * a.B * a.C * a.C * a.T * 8
    nb = 4.0 * x_act.numel() * (3 + a.dual - a.lazy)
    print(f"resunit C={a.C} d={a.d} T={a.T} B={a.B} dual={int(a.dual)} cfg={cfg} ({L.resunit_kernel_name(cfg, a.C, a.d)}) "
          f"rr={os.environ.get('BC_RU_RR', '1')} lazy={int(a.lazy)}: {ms:.3f} ms  {fl / ms / 1e9:.1f} TFLOP/s  {nb / ms / 1e6:.0f} GB/s",
          flush=True)


if __name__ == "__main__":
    main()
