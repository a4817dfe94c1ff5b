"""Run-to-run determinism probe of the full-size encoder (x6 latent off by 5.1e-4 on a fresh box).

Every precision of the HIP path has a fixed accumulation order, so two forwards of the same batch must be bit-identical;
a difference localises a race.  The probe runs the config-2 batch (64 x 240 000, default model) through the encoder stage
by stage, first in h3 (to leave h3 data in every reused workspace, as the GPU test order does), then R times in each
requested precision, and reports per stage whether the output equals the first repeat bit for bit, and the latent of
clip 0 against the reference fixture.

usage: python tools/lab/x6_race_probe.py [--repeats 6] [--precisions x6,h3]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from helpers import build_models, max_rel_err  # noqa: E402

from audiotokenization_amd import _lib  # noqa: E402
from audiotokenization_amd.blocks import EncoderBlock, input_act, produce_conv  # noqa: E402
from audiotokenization_amd.extract import synth_batch  # noqa: E402


def staged(enc, x):
    """BigCodecEncoder.forward (codec.py:53-74) with every stage's output kept."""
    blk = list(enc.block)
    final_act, last_conv = blk[-2], blk[-1]
    stages = blk[1:-2]

    def next_act_of(i):
        if i + 1 < len(stages):
            nxt = stages[i + 1]
            return input_act(nxt) if isinstance(nxt, EncoderBlock) else None
        return final_act
    outs = []
    y, ya = produce_conv(blk[0], x, None, want_raw=True, next_act=next_act_of(-1))
    outs.append(("conv0", y if y is not None else ya))
    for i, st in enumerate(stages):
        nact = next_act_of(i)
        want_raw = i + 1 < len(stages)
        if isinstance(st, EncoderBlock):
            y, ya = st.flow(y, ya, want_raw=want_raw, next_act=nact)
            outs.append((f"block{i}", y if y is not None else ya))
        else:
            y, ya = st.flow(y, want_raw=want_raw, next_act=nact)
            outs.append(("reslstm", y if y is not None else ya))
    out = produce_conv(last_conv, ya, None, want_raw=True, next_act=None)[0]
    _lib.check_status()
    outs.append(("latent", out))
    return outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeats", type=int, default=6)
    ap.add_argument("--precisions", default="x6,h3")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    _lib.load()
    g = np.load(os.path.join(REPO, "tests", "golden", "full_config2_default.npz"), allow_pickle=False)
    enc = build_models("default", device=dev)[0]
    x = synth_batch(64, 240000, 0, dev)
    with torch.no_grad():
        _lib.set_precision("h3")
        staged(enc, x)
        torch.cuda.synchronize()
        bad_total = 0
        for prec in args.precisions.split(","):
            _lib.set_precision(prec)
            first = None
            for r in range(args.repeats):
                t0 = time.time()
                outs = staged(enc, x)
                torch.cuda.synchronize()
                lat0 = outs[-1][1][0].cpu().numpy()
                err = max_rel_err(lat0, g["latent0"])
                line = [f"[{prec}] repeat {r}: {time.time() - t0:.2f} s, latent clip 0 vs reference {err:.2e}"]
                if first is None:
                    first = [(n, t.clone()) for n, t in outs]
                else:
                    for (n, t), (_, t0_) in zip(outs, first):
                        if not torch.equal(t, t0_):
                            d = (t - t0_).abs()
                            nz = (d > 0).nonzero()
                            line.append(f"  {n}: DIFFERS, {nz.shape[0]} elements, max {float(d.max()):.2e}, first at "
                                        f"{nz[0].tolist()}, frames {int(nz[:, -1].min())}..{int(nz[:, -1].max())}")
                            bad_total += 1
                print("\n".join(line), flush=True)
            del first
            torch.cuda.empty_cache()
    print(f"probe done: {bad_total} stage outputs differed from their first repeat")
    return 1 if bad_total else 0


if __name__ == "__main__":
    sys.exit(main())
