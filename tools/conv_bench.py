"""Time one conv shape on the GPU for a list of tile cfgs (HIP events, warm, back to back).

    python tools/conv_bench.py --cin 384 --cout 384 --k 1 --T 30000 --B 64 --res --snake --dual \
        [--cfg 117,100] [--iters 10]

Without --cfg the library's own choice (bc_conv1d_select_cfg) is timed.  Prints ms per launch,
fp32-equivalent TFLOP/s and the algorithmic HBM GB/s (input + output [+ residual, + dual]).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# BIGCODEC_PKG_ROOT: import the package from another tree (e.g. an ablation build, tools/lab/r03h_ablation.sh)
sys.path.insert(0, os.environ.get("BIGCODEC_PKG_ROOT", REPO))

import torch  # noqa: E402

from audiotokenization_amd import _lib as L  # noqa: E402
from audiotokenization_amd import conv as CV  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--cin", type=int, required=True)
    p.add_argument("--cout", type=int, required=True)
    p.add_argument("--k", type=int, default=1)
    p.add_argument("--s", type=int, default=1)
    p.add_argument("--d", type=int, default=1)
    p.add_argument("--T", type=int, default=30000, help="output length")
    p.add_argument("--B", type=int, default=64)
    p.add_argument("--res", action="store_true")
    p.add_argument("--snake", action="store_true")
    p.add_argument("--dual", action="store_true")
    p.add_argument("--cfg", default="")
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--precision", default="x6")
    a = p.parse_args()
    L.set_precision(a.precision)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    pad = (a.k - 1) * a.d // 2
    m = CV.Conv1dWN(a.cin, a.cout, a.k, stride=a.s, dilation=a.d, padding=pad)
    with torch.no_grad():
        m.weight_v.copy_(torch.randn(m.weight_v.shape, generator=g))
        if m.bias is not None:
            m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)
    Tin = (a.T - 1) * a.s + (a.k - 1) * a.d + 1 - 2 * pad
    x = torch.randn(a.B, a.cin, Tin, generator=g).to(dev)
    Tout = m.out_len(Tin)
    y = torch.empty(a.B, a.cout, Tout, device=dev)
    y2 = torch.empty_like(y) if a.dual else None
    res = torch.randn(a.B, a.cout, Tout, generator=g).to(dev) if a.res else None
    sa = torch.rand(a.cout, generator=g).to(dev) + 0.5 if (a.snake or a.dual) else None
    sb = torch.rand(a.cout, generator=g).to(dev) + 0.5 if (a.snake or a.dual) else None
    lib = L.load()
    chosen = lib.bc_conv1d_select_cfg(a.cout, a.cin, a.k, a.s, a.d, L.precision_mode())
    if a.cfg == "all":  # every x6 tile (and, for stride >= 2, every phase-decomposed one)
        base = {"x6": 0, "bf16": 100, "h3": 200}[a.precision]
        tiles = [c + base for c in sorted(L.X6_CFGS)]
        cfgs = tiles + ([1000 * a.s + c for c in tiles] if a.s >= 2 else [])
    else:
        cfgs = [chosen if c == "c" else int(c) for c in a.cfg.split(",") if c] or [chosen]  # "c": the library's
    st = torch.cuda.current_stream().cuda_stream
    fl = 2.0 * a.B * a.cout * a.cin * a.k * Tout
    nb = 4.0 * (x.numel() + y.numel() * (1 + a.res + a.dual))
    best = None
    for cfg in cfgs:
        wp, bias = m.packed_as(cfg, dev)

        def run():
            L.call("bc_conv1d_fwd", x.data_ptr(), wp.data_ptr(), L.ptr(bias), L.ptr(res), L.ptr(sa), L.ptr(sb),
                   y.data_ptr(), L.ptr(y2), a.B, a.cin, Tin, a.cout, Tout, a.k, a.s, a.d, pad, 0, cfg, st)

        try:
            run()
        except L.BigCodecLibraryError as e:
            if "unsupported" in str(e):
                continue
            raise
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        best = min(best or (ms, cfg), (ms, cfg))
        print(f"Cin={a.cin} Cout={a.cout} k={a.k} s={a.s} d={a.d} T={Tout} B={a.B} cfg={cfg}{'*' if cfg == chosen else ''} "
              f"({L.conv_kernel_name(cfg, a.k, a.s, a.d)}): {ms:.3f} ms  {fl / ms / 1e9:.1f} TFLOP/s  "
              f"{nb / ms / 1e6:.0f} GB/s", flush=True)
    if len(cfgs) > 1 and best:
        print(f"  best cfg {best[1]} {best[0]:.3f} ms (library choice {chosen})", flush=True)


if __name__ == "__main__":
    main()
