"""Causal streaming throughput on the GPU: a causal `default` BigCodec encoder (and decoder) fed chunk by chunk.

    python tools/stream_bench.py [--B 64] [--seconds 10] [--chunk 12000] [--prev] [--decode]

Prints audio-seconds per second of the stream (every chunk of a B-clip batch pushed back to back, HIP-synchronised
around the whole stream), ms per push and the number of kernel launches per push (rocprofv3 gives the names).
--graph replays one captured HIP graph per chunk (StreamGraph; status words read once at the end).
--prev times the round-4 first-session stream (tools/lab/streaming_prev.py: separate Snake launches, torch.cat
contexts, two-launch ResidualUnits) on the same models for an A/B.  Random weights, synthetic white noise.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools", "lab"))

import torch  # noqa: E402

from audiotokenization_amd import config, synth  # noqa: E402
from audiotokenization_amd.codec import BigCodecDecoder, BigCodecEncoder  # noqa: E402
from audiotokenization_amd.extract import synth_batch  # noqa: E402


def build_model_pair(name, device, **ov):
    """Encoder / decoder of preset `name` with synthetic weights (bench.py's build_model)."""
    cfg = config.preset(name, **ov)
    enc = BigCodecEncoder(**config.encoder_kwargs(cfg.model.codec_encoder))
    dec = BigCodecDecoder(**config.decoder_kwargs(cfg.model.codec_decoder))
    for m, prefix in ((enc, "encoder."), (dec, "decoder.")):
        syn = synth.synth_state_dict({prefix + k: v for k, v in m.state_dict().items()})
        m.load_state_dict({k[len(prefix):]: torch.from_numpy(v) for k, v in syn.items()}, strict=True)
    return enc.eval().to(device), dec.eval().to(device)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--B", type=int, default=64)
    p.add_argument("--seconds", type=float, default=10.0)
    p.add_argument("--chunk", type=int, default=12000, help="samples per push (encode) / x hop (decode)")
    p.add_argument("--prev", action="store_true")
    p.add_argument("--decode", action="store_true")
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--graph", action="store_true", help="push through a StreamGraph (one HIP-graph replay per chunk)")
    a = p.parse_args()
    if a.prev:
        import streaming_prev as S
    else:
        from audiotokenization_amd import streaming as S
    dev = torch.device("cuda:0")
    enc, dec = build_model_pair("default", device=dev, causal=True)
    n = int(a.seconds * 24000) // 200 * 200
    x = synth_batch(a.B, n, 0, dev)
    with torch.no_grad():
        if a.decode:
            z = dec(enc(x), vq=True)[0]
            s = S.StreamingDecoder(dec)
            step = a.chunk // 200
            data, width = z, step
        else:
            s = S.StreamingEncoder(enc)
            data, width = x, a.chunk
        best = None
        g = s.graph(data[..., :width]) if a.graph else None
        if g is not None and data.shape[-1] % width:
            raise SystemExit("--graph needs the stream length to be a multiple of the chunk")
        for _ in range(a.reps + 1):
            s.reset() if g is None else g.reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pushes = 0
            for i in range(0, data.shape[-1], width):
                if g is not None:
                    g.push(data[..., i:i + width], check=False)
                else:
                    s.push(data[..., i:i + width])
                pushes += 1
            if g is not None:
                g.check()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
    what = "decode" if a.decode else "encode"
    mode = "prev" if a.prev else ("graph" if a.graph else "current")
    print(f"stream {what} ({mode}): B {a.B} x {n / 24000:.1f} s, chunk {a.chunk} samples, "
          f"{pushes} pushes: {a.B * n / 24000 / best:.1f} audio-s/s, {1e3 * best / pushes:.2f} ms per push")


if __name__ == "__main__":
    main()
