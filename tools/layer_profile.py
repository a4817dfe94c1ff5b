"""Per-launch timing of one encode+VQ step (HIP events on the launch stream), grouped by layer
shape: where the time goes and at what TFLOP/s each conv runs.

    python tools/layer_profile.py [--model default] [--batch 64] [--seconds 10]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from audiotokenization_amd import _lib as L  # noqa: E402
from audiotokenization_amd import modules as M  # noqa: E402
from audiotokenization_amd.extract import synth_batch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="default")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--seconds", type=float, default=10.0)
    p.add_argument("--precision", default="h3")
    p.add_argument("--decode", action="store_true", help="profile the decoder (dec(z_q, vq=False)) instead of encode + VQ")
    a = p.parse_args()
    L.set_precision(a.precision)
    import bench

    dev = torch.device("cuda", 0)
    enc, dec, *_ = bench.build_model(a.model, dev)
    x = synth_batch(a.batch, int(a.seconds * 24000), 0, dev)
    rows = []
    from audiotokenization_amd import blocks as BLK
    from audiotokenization_amd import conv as CV
    orig = CV.Conv1dWN.run

    def timed_run(self, x, residual=None, epilogue=0, out_snake=None, dual=False):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig(self, x, residual, epilogue, out_snake, dual)
        y = out[0] if dual else out
        e1.record()
        B, Cin, T = x.shape
        fl = 2.0 * B * self.out_channels * Cin * self.kernel_size * y.shape[-1]
        rows.append((f"conv Cin={Cin} Cout={self.out_channels} k={self.kernel_size} s={self.stride} "
                     f"d={self.dilation} T={y.shape[-1]}{' snake' if out_snake is not None else ''}{' res' if residual is not None else ''}",
                     fl, e0, e1))
        return out

    lorig = BLK.ResLSTM.run

    def timed_lstm(self, x, out_snake=None):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        y = lorig(self, x, out_snake)
        e1.record()
        B, H, T = x.shape
        fl = 2.0 * 2 * B * T * 4 * H * H * self.lstm.num_layers
        rows.append((f"ResLSTM H={H} T={T} layers={self.lstm.num_layers}", fl, e0, e1))
        return y

    torig = CV.ConvTranspose1dWN.run

    def timed_convt(self, x, out_snake=None, dual=False):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out = torig(self, x, out_snake, dual)
        y = out[0] if dual else out
        e1.record()
        B, Cin, T = x.shape
        fl = 2.0 * B * self.out_channels * Cin * self.kernel_size * T
        rows.append((f"convT Cin={Cin} Cout={self.out_channels} k={self.kernel_size} s={self.stride} T={y.shape[-1]}"
                     f"{' snake' if out_snake is not None else ''}", fl, e0, e1))
        return out

    rorig = BLK.ResidualUnit._flow_fused

    def timed_ru(self, cfg, x_raw, x_act, want_raw, next_act):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out = rorig(self, cfg, x_raw, x_act, want_raw, next_act)
        e1.record()
        B, C, T = x_raw.shape
        conv7 = BLK._conv_of(self.block[1])
        rows.append((f"resunit C={C} d={conv7.dilation} T={T}{' dual' if want_raw and next_act else ''}",
                     2.0 * B * C * C * T * 8, e0, e1))
        return out

    with torch.no_grad():
        zq = dec(enc(x), vq=True)[0]  # warm-up / weight prep
        if a.decode:
            dec(zq, vq=False)
        torch.cuda.synchronize()
        CV.Conv1dWN.run = timed_run
        CV.ConvTranspose1dWN.run = timed_convt
        BLK.ResLSTM.run = timed_lstm
        BLK.ResidualUnit._flow_fused = timed_ru
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        if a.decode:
            dec(zq, vq=False)
        else:
            dec(enc(x), vq=True)
        e1.record()
        torch.cuda.synchronize()
    total = e0.elapsed_time(e1)
    agg = {}
    for name, fl, a0, a1 in rows:
        d = agg.setdefault(name, [0, 0.0, 0.0])
        d[0] += 1
        d[1] += a0.elapsed_time(a1)
        d[2] += fl
    print(f"step {total:.1f} ms")
    for name, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{ms:9.2f} ms {100 * ms / total:5.1f}%  x{n}  {fl / ms / 1e9:7.1f} TFLOP/s  {name}")


if __name__ == "__main__":
    main()
