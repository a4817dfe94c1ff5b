"""Time one ResLSTM layer stack on the GPU (the recurrence dominates at T = 1200).

    python tools/lstm_bench.py [--H 1536] [--B 64] [--T 1200] [--layers 1] [--precision x6]

BC_LSTM_SEQ_DEBUG (read once per process by the library) switches parts of the persistent kernel
off for timing experiments: 1 = no MFMA, 2 = no h loads, 4 = no flag poll (results are garbage).
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from audiotokenization_amd import _lib as L  # noqa: E402
from audiotokenization_amd import blocks as BL  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--H", type=int, default=1536)
    p.add_argument("--B", type=int, default=64)
    p.add_argument("--T", type=int, default=1200)
    p.add_argument("--layers", type=int, default=1)
    p.add_argument("--precision", default="x6")
    p.add_argument("--iters", type=int, default=3)
    a = p.parse_args()
    L.set_precision(a.precision)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    m = BL.ResLSTM(a.H, num_layers=a.layers)
    with torch.no_grad():
        for prm in m.lstm.parameters():
            prm.copy_((torch.rand(prm.shape, generator=g) * 2 - 1) / np.sqrt(a.H))
    m.to(dev)
    x = torch.randn(a.B, a.H, a.T, generator=g).to(dev)
    with torch.no_grad():
        m.run(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            m.run(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
    st = L.load().bc_lstm_status(1)
    print(f"H={a.H} B={a.B} T={a.T} layers={a.layers} prec={a.precision} "
          f"dbg={os.environ.get('BC_LSTM_SEQ_DEBUG', '0')}: {dt * 1e3:.2f} ms "
          f"({dt * 1e6 / (a.T * a.layers):.2f} us/step incl. input projection) status={st}", flush=True)
    if os.environ.get("BC_LSTM_SEQ_STAMPS"):
        timeline(a.T)


def timeline(T):
    """Per-step phase durations (s_memtime ticks) of workgroups 0 and G/2 from the last launch:
    0 step start, 1 poll done, 2 MFMAs done, 3 reduction barrier passed, 4 cell done,
    5 gather barrier passed, 6 publish done (wave 0)."""
    import ctypes as C

    lib = L.load()
    n = 2 * 2048 * 32
    buf = (C.c_longlong * n)()
    fn = lib.bc_debug_lstm_stamps
    fn.argtypes = [C.c_void_p, C.c_longlong]
    if fn(C.addressof(buf), n) != 0:
        print("no stamps")
        return
    if os.environ.get("BC_LSTM_SEQ_HALVES", "2") != "1":
        T = min(2048, 2 * T)  # rows are half-steps (2t + half)
        print("rows = half-steps")
    s = np.frombuffer(buf, dtype=np.int64).reshape(2, 2048, 4, 8)[:, :T]
    names = ["poll", "load+mfma", "red.barrier", "cell", "gather.barrier", "publish", "tail->next"]
    lo, hi = 10, T - 10
    for wgi in range(2):
        step = s[wgi, lo + 1:hi + 1, 0, 0] - s[wgi, lo:hi, 0, 0]
        print(f"workgroup {'0' if wgi == 0 else 'G/2'}: step {np.median(step):.0f} ticks (median)")
        for w in range(4):
            d = [np.median(s[wgi, lo:hi, w, k + 1] - s[wgi, lo:hi, w, k]) for k in range(6)]
            d.append(np.median(s[wgi, lo + 1:hi + 1, w, 0] - s[wgi, lo:hi, w, 6]))
            print(f"  wave {w}: " + "  ".join(f"{nm} {v:6.0f}" for nm, v in zip(names, d)))


if __name__ == "__main__":
    main()
