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


if __name__ == "__main__":
    main()
