"""Benchmark: BASELINE.json config 2 — batch = 64 x 10 s @24 kHz clips, encode + VQ (the
extract_indices.py path: encoder -> decoder(vq=True) -> codes) of the `default` BigCodec model on each
GPU, fp32, synthetic white-noise clips already resident in HBM, random (counter-hash) weights.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model default] [--batch 64]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

A step = one batch per GPU through the hot path; for N > 1 each step ends with the RCCL all-gather
of the batch's index tensor (clip-sharded data parallelism, weak scaling).  Rank 0 prints one JSON
line with the whole-job throughput (audio-seconds encoded per second, all GPUs), the roofline of
the dominant kernel (HIP-event timed inside the timed region) and the CPU oracle baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "audio-sec encoded/sec/GPU (24 kHz mono, 10 s clips) + VQ index bit-exactness"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix peak (spec); 155 measured
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (no sparsity)
X6_PRODUCTS = 6  # csrc/conv1d_x6.hip: six bf16 MFMAs per fp32-accurate product term
HBM_PEAK_GBS = 8000.0


def kernel_peak(kname: str):
    """(peak in fp32-equivalent TFLOP/s, MFMA instructions per algorithmic FLOP pair, note)."""
    if kname.startswith("conv1d_x6_kernel"):
        return (BF16_MFMA_PEAK_TFLOPS / X6_PRODUCTS, X6_PRODUCTS,
                "3xbf16 split: every fp32 multiply-add costs 6 bf16 MFMA multiply-adds, so the fp32-equivalent "
                "ceiling is the dense BF16 MFMA peak / 6")
    return FP32_MFMA_PEAK_TFLOPS, 1, "native fp32 MFMA peak"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="default")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--seconds", type=float, default=10.0)
    p.add_argument("--sample-rate", type=int, default=24000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-timer", action="store_true")
    p.add_argument("--cpu-clips", type=int, default=1)
    p.add_argument("--precision", choices=["fp32", "x6"], default=None,
                   help="conv GEMM arithmetic (default: BIGCODEC_PRECISION or x6)")
    return p.parse_args()


def build_model(name, device):
    import torch

    from audiotokenization_amd import config, synth
    from audiotokenization_amd.codec import BigCodecDecoder, BigCodecEncoder

    cfg = config.preset(name)
    ek = config.encoder_kwargs(cfg.model.codec_encoder)
    dk = config.decoder_kwargs(cfg.model.codec_decoder)
    enc, dec = BigCodecEncoder(**ek), BigCodecDecoder(**dk)
    sds = []
    for m, prefix in ((enc, "encoder."), (dec, "decoder.")):
        full = {prefix + k: v for k, v in m.state_dict().items()}
        syn = synth.synth_state_dict(full)
        local = {k[len(prefix):]: torch.from_numpy(v) for k, v in syn.items()}
        m.load_state_dict(local, strict=True)
        sds.append(local)
    enc.eval().to(device)
    dec.eval().to(device)
    return enc, dec, sds, ek, dk


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (tools/gpu_pmc.sh ->
    tools/pmc_summary.py -> profiles/*pmc_traffic.json), or (None, None)."""
    import glob

    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))["kernels"].get(kernel)
    if not d:
        return None, None
    return d["traffic_bytes_corrected"], os.path.basename(files[-1])


def cpu_baseline(name, n_samples, sds, ek, dk, n_clips):
    """The CPU oracle (torch CPU restatement, bit-identical to the reference in the development
    container) timed on this host: encode + VQ, B = 1 per clip (extract_indices.py:397), warm run."""
    import torch

    from audiotokenization_amd import synth
    from oracle import bigcodec_oracle as O

    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    torch.set_num_threads(threads)
    x = torch.from_numpy(synth.synth_clips(n_clips, n_samples, clip0=0)).unsqueeze(1)
    codes = []
    with torch.no_grad():
        O.encode_indices(x[:1, :, : n_samples // 10], sds[0], sds[1], ek, dk)  # warm-up (short)
        t0 = time.perf_counter()
        for i in range(n_clips):
            c, _ = O.encode_indices(x[i:i + 1], sds[0], sds[1], ek, dk)
            codes.append(c)
        dt = time.perf_counter() - t0
    audio_s = n_clips * n_samples / 24000.0
    return dict(value=audio_s / dt, unit="audio-sec/s", cores=threads, kind="port",
                sample=f"{n_clips} clip(s) x {n_samples / 24000:.0f} s @24 kHz, {name} model, encode+VQ, B=1 "
                       f"(extract_indices.py:397), torch CPU oracle, {dt:.1f} s"), torch.cat(codes, dim=1)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from audiotokenization_amd import _lib
    from audiotokenization_amd.extract import all_gather_codes, synth_batch

    _lib.load()
    if args.precision:
        _lib.set_precision(args.precision)
    args.precision = _lib.precision_name()
    n_samples = int(round(args.seconds * args.sample_rate))
    enc, dec, sds, ek, dk = build_model(args.model, dev)
    B = args.batch
    x = synth_batch(B, n_samples, clip0=rank * B, device=dev)  # resident in HBM before timing

    def step():
        with torch.no_grad():
            codes = dec(enc(x), vq=True)[1]
            if world > 1:
                codes = all_gather_codes(codes)
        return codes

    for _ in range(args.warmup):
        codes = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timer = None if args.no_kernel_timer else _lib.KernelTimer()
    _lib.set_timer(timer)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        codes = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    _lib.set_timer(None)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    audio_s = world * B * n_samples / args.sample_rate * args.steps
    value = audio_s / elapsed
    roof = None
    if timer is not None:
        summ = timer.summary()
        kname, d = max(summ.items(), key=lambda kv: kv[1]["ms_total"])
        avg_ms = d["ms_total"] / d["launches"]
        achieved = d["flops_total"] / d["launches"] / (avg_ms * 1e-3) / 1e12
        conv_ms = sum(v["ms_total"] for v in summ.values())
        traffic, tsrc = pmc_traffic(kname)
        peak, mult, note = kernel_peak(kname)
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "peak_note": note,
                "mfma_tflops_executed": round(achieved * mult, 2),
                "traffic": round(traffic) if traffic else None, "traffic_source": tsrc,
                "algorithmic_bytes_per_launch": round(d["bytes_total"] / d["launches"]), "kernel": kname,
                "launches_per_step": d["launches"] // args.steps, "avg_launch_ms": round(avg_ms, 4),
                "algorithmic_gflop_per_launch": round(d["flops_total"] / d["launches"] / 1e9, 3),
                "all_python_conv_kernels_ms_per_step": round(conv_ms / args.steps, 2),
                "all_python_conv_tflops": round(sum(v["flops_total"] for v in summ.values()) / (conv_ms * 1e-3) / 1e12, 2)}

    cpu = None
    parity = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu, codes_ref = cpu_baseline(args.model, n_samples, sds, ek, dk, args.cpu_clips)
        got = codes[0] if world > 1 else codes
        got = got[:, : args.cpu_clips].cpu()
        parity = {"clips_checked": args.cpu_clips, "frames": int(got.numel()),
                  "index_mismatches": int((got != codes_ref).sum())}
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "audio-sec/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" if args.precision == "fp32" else "f32 (3xbf16-split MFMA, fp32 accumulate)",
            "data": "synthetic",
            "config": {"workload": f"config2: batch={B} x {args.seconds:g} s {args.sample_rate // 1000} kHz clips per GPU, "
                                   f"encode+VQ (extract_indices path), BigCodec '{args.model}' model, random weights",
                       "global_batch": B * world, "clip_samples": n_samples, "parallelism": f"dp{world}"},
            "roofline": roof, "cpu_baseline": cpu, "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
