"""Benchmark of the BigCodec tokenization hot path on MI355X (BASELINE.json configs).

Default (what the driver runs) = BASELINE config 2: batch = 64 x 10 s @24 kHz clips per GPU, encode +
VQ (the extract_indices.py path: encoder -> decoder(vq=True) -> codes) of the `default` BigCodec
model, fp32-accurate arithmetic, synthetic white-noise clips already resident in HBM, random
(counter-hash) weights.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--precision fp32|x6|bf16]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

--config 3: full encode -> VQ -> decode round trip (inference_full.py's model path), parity adds the
            decoder's waveform error against the CPU oracle decoding the same codes.
--config 4: extract_indices-style corpus streaming: every step synthesises the rank's NEXT batch of
            clips on the device, encodes + quantises it, all-gathers the indices (RCCL) and copies
            them to the host as int16 (the .npy payload).
--config 5: batch = 32 x 30 s per GPU with bf16 conv products (precision 'bf16'); parity reports the
            index mismatch rate against the fp32-accurate path on the same batch.

A step = one batch per GPU through the path; for N > 1 each step ends with the RCCL all-gather of the
batch's index tensor (clip-sharded data parallelism, weak scaling).  Rank 0 prints one JSON line with
the whole-job throughput (audio-seconds per second, all GPUs), the roofline of the dominant kernel
(HIP-event timed inside the timed region) and the CPU oracle baseline.
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
METRIC_RT = "audio-sec encoded+quantised+decoded/sec (24 kHz mono, 10 s clips)"
METRIC_DEC = "audio-sec decoded from tokens/sec/GPU (24 kHz mono, 10 s clips)"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix peak (spec); 155 measured
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 MFMA ~2.5 PF dense (no sparsity)
H3_PRODUCTS = 3  # csrc/conv1d_x6.hip P = 2: three fp16 MFMAs per product term
X6_PRODUCTS = 6  # csrc/conv1d_x6.hip: six bf16 MFMAs per fp32-accurate product term
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    2: dict(batch=64, seconds=10.0, precision=None, work="encode+VQ (extract_indices path)"),
    3: dict(batch=64, seconds=10.0, precision=None, work="encode+VQ+decode round trip (inference_full path)"),
    4: dict(batch=64, seconds=10.0, precision=None,
            work="corpus streaming: on-device clip synthesis + encode+VQ + index all-gather + int16 host copy"),
    5: dict(batch=32, seconds=30.0, precision="bf16", work="encode+VQ, bf16 conv products"),
    6: dict(batch=64, seconds=10.0, precision=None,
            work="token -> audio: (B, F, 1) int64 codes resident in HBM -> bc_vq2emb_ct -> decoder "
                 "(tokens.py service path, SURVEY 8(f) rank 3)"),
}


def kernel_peak(kname: str):
    """(peak in fp32-equivalent TFLOP/s, MFMA instructions per algorithmic FLOP pair, note)."""
    targs = [t.strip() for t in kname[kname.find("<") + 1:kname.rfind(">")].split(",")] if "<" in kname else []
    planes = targs[4] if kname.startswith(("conv1d_x6_kernel", "resunit_x6_kernel")) and len(targs) >= 5 else None
    if planes == "1":
        return BF16_MFMA_PEAK_TFLOPS, 1, "bf16 products (precision 'bf16'): dense BF16 MFMA peak"
    if planes == "2":
        return (BF16_MFMA_PEAK_TFLOPS / H3_PRODUCTS, H3_PRODUCTS,
                "2xfp16 split (h3): every fp32 multiply-add costs 3 fp16 MFMA multiply-adds (dense FP16 MFMA peak "
                "= BF16's), so the fp32-equivalent ceiling is the dense FP16 MFMA peak / 3")
    if planes == "3":
        return (BF16_MFMA_PEAK_TFLOPS / X6_PRODUCTS, X6_PRODUCTS,
                "3xbf16 split: every fp32 multiply-add costs 6 bf16 MFMA multiply-adds, so the fp32-equivalent "
                "ceiling is the dense BF16 MFMA peak / 6")
    return FP32_MFMA_PEAK_TFLOPS, 1, "native fp32 MFMA peak"


def kernel_table(summ, steps, probe, n=8):
    """The n most time-consuming HIP-event-timed kernels of the timed steps: ms per step, algorithmic
    TFLOP/s against the kernel's MFMA ceiling (spec and probe-measured) and algorithmic GB/s against
    the 8 TB/s HBM peak.  The kernels' rows are the ones bench's roofline entry is drawn from."""
    rows = []
    for name, d in sorted(summ.items(), key=lambda kv: -kv[1]["ms_total"])[:n]:
        sec = d["ms_total"] * 1e-3
        tf = d["flops_total"] / sec / 1e12
        peak, mult, _ = kernel_peak(name)
        gbs = d["bytes_total"] / sec / 1e9
        rows.append({"kernel": name, "launches_per_step": d["launches"] // steps,
                     "ms_per_step": round(d["ms_total"] / steps, 3), "tflops": round(tf, 1),
                     "frac_mfma_spec": round(tf / peak, 3),
                     "frac_mfma_probe": round(tf * mult / probe, 3) if name.startswith(("conv1d_x6", "resunit_x6")) else None,
                     "gbs": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 3)})
    return rows


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    p.add_argument("--model", default="default")
    p.add_argument("--batch", type=int, default=None, help="clips per GPU (default: the config's)")
    p.add_argument("--seconds", type=float, default=None, help="clip length (default: the config's)")
    p.add_argument("--sample-rate", type=int, default=24000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-timer", action="store_true")
    p.add_argument("--cpu-clips", type=int, default=4, help="clips in the CPU-baseline sample (about 3 s each)")
    p.add_argument("--precision", choices=["fp32", "x6", "bf16", "h3"], default=None,
                   help="conv GEMM arithmetic (default: the config's, else BIGCODEC_PRECISION or h3)")
    a = p.parse_args()
    c = CONFIGS[a.config]
    a.batch = a.batch or c["batch"]
    a.seconds = a.seconds or c["seconds"]
    a.precision = a.precision or c["precision"]
    return a


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
    """(HBM bytes per launch, MFMA utilisation, source file) of `kernel` from the newest committed PMC
    summary (tools/gpu_pmc.sh -> tools/pmc_summary.py -> profiles/*pmc_traffic.json), or Nones."""
    import glob

    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_traffic.json")))  # r01_ < r01a_ < ... < r01h_
    for f in reversed(files):
        d = json.load(open(f))["kernels"].get(kernel)
        if d:
            return d["traffic_bytes_corrected"], d.get("mfma_util"), os.path.basename(f)
    return None, None, None


def mfma_probe_tflops(dev, nwg=2048, iters=60000):
    """Dense BF16 MFMA rate this device sustains on random register operands (bc_mfma_probe: no
    memory, four waves per SIMD on every CU), in TFLOP/s: the practical ceiling under the chip's
    clock management, beside the 2.5 PFLOP/s spec peak (MI355X_MICROARCH.md 'DVFS give-back')."""
    import torch

    from audiotokenization_amd import _lib

    out = torch.empty(nwg * 4, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    _lib.call("bc_mfma_probe", out.data_ptr(), nwg, iters // 3, st)  # warm, clock settles
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.call("bc_mfma_probe", out.data_ptr(), nwg, iters, st)
    e1.record()
    torch.cuda.synchronize()
    return nwg * 4 * iters * 16 * 16384.0 / (e0.elapsed_time(e1) * 1e-3) / 1e12


def cpu_baseline(name, n_samples, sds, ek, dk, n_clips, roundtrip=False):
    """The CPU oracle (torch CPU restatement, bit-identical to the reference in the development
    container) timed on this host: encode + VQ (+ decode for the round trip), B = 1 per clip
    (extract_indices.py:397), warm run.  Returns (baseline dict, codes, waveforms or None)."""
    import torch

    from audiotokenization_amd import synth
    from oracle import bigcodec_oracle as O

    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    torch.set_num_threads(threads)
    x = torch.from_numpy(synth.synth_clips(n_clips, n_samples, clip0=0)).unsqueeze(1)
    codes, wavs = [], []
    with torch.no_grad():
        O.encode_indices(x[:1, :, : n_samples // 10], sds[0], sds[1], ek, dk)  # warm-up (short)
        t0 = time.perf_counter()
        for i in range(n_clips):
            c, emb = O.encode_indices(x[i:i + 1], sds[0], sds[1], ek, dk)
            codes.append(c)
            if roundtrip:
                zq, _, _ = O.rvq_forward(emb, sds[1], "quantizer.", dk.get("vq_num_quantizers", 1))
                wavs.append(O.decoder_forward(zq, sds[1], dk))
        dt = time.perf_counter() - t0
        # also the batched CPU rate (the same clips as one B = n_clips call); best of both
        dtb = None
        if not roundtrip and n_clips > 1:
            t0 = time.perf_counter()
            O.encode_indices(x, sds[0], sds[1], ek, dk)
            dtb = time.perf_counter() - t0
    audio_s = n_clips * n_samples / 24000.0
    what = "encode+VQ+decode" if roundtrip else "encode+VQ"
    rates = {"B=1": audio_s / dt}
    if dtb:
        rates[f"B={n_clips}"] = audio_s / dtb
    best = max(rates, key=rates.get)
    return (dict(value=rates[best], unit="audio-sec/s", cores=threads, kind="port", rates=rates,
                 sample=f"{n_clips} clip(s) x {n_samples / 24000:.0f} s @24 kHz, {name} model, {what}, best of "
                        f"{'/'.join(rates)} ({best}; B=1 is extract_indices.py:397), torch CPU oracle, "
                        f"{dt + (dtb or 0):.1f} s"),
            torch.cat(codes, dim=1), torch.cat(wavs, dim=0) if roundtrip else None)


def cpu_decode_baseline(codes, sds, dk, n_clips):
    """The CPU oracle's token -> audio decode (vq2emb -> transpose -> decoder) on this host, B = 1 per
    clip, warm.  Returns (baseline dict, waveforms)."""
    import numpy as np
    import torch

    from oracle import bigcodec_oracle as O

    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    torch.set_num_threads(threads)
    nq = codes.shape[2]
    with torch.no_grad():
        O.decoder_forward(O.vq2emb(codes[:1, :20], sds[1], "quantizer.", nq).transpose(1, 2).contiguous(), sds[1], dk)
        wavs = []
        t0 = time.perf_counter()
        for i in range(n_clips):
            emb = O.vq2emb(codes[i:i + 1], sds[1], "quantizer.", nq)
            wavs.append(O.decoder_forward(emb.transpose(1, 2).contiguous(), sds[1], dk))
        dt = time.perf_counter() - t0
    audio_s = n_clips * codes.shape[1] * int(np.prod(dk["up_ratios"])) / 24000.0
    return (dict(value=audio_s / dt, unit="audio-sec/s", cores=threads, kind="port",
                 sample=f"{n_clips} clip(s) x {codes.shape[1]} frames, token -> audio decode, B=1, torch CPU "
                        f"oracle, {dt:.1f} s"),
            torch.cat(wavs, dim=0))


def main():
    args = parse()
    import numpy as np
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
    from audiotokenization_amd.extract import all_gather_codes, batch_indices_to_numpy, synth_batch

    _lib.load()
    if args.precision:
        _lib.set_precision(args.precision)
    args.precision = _lib.precision_name()
    n_samples = int(round(args.seconds * args.sample_rate))
    enc, dec, sds, ek, dk = build_model(args.model, dev)
    B = args.batch
    cfgn = args.config
    x = synth_batch(B, n_samples, clip0=rank * B, device=dev)  # resident in HBM before timing
    state = {"batch": 0, "wav": None, "host": None}
    tok = None
    if cfgn == 6:  # synthetic codes of the clips' frame count, uniform over the codebook, seeded per rank
        n_frames = n_samples // int(dec.hop_length)
        g = torch.Generator().manual_seed(1234 + rank)
        tok = torch.randint(0, dec.quantizer.layers[0].codebook_size, (B, n_frames, 1), generator=g)
        tok_dev = tok.to(dev)

    def step():
        if cfgn == 6:
            with torch.no_grad():
                state["wav"] = dec.tokens_to_audio(tok_dev)
            return None
        with torch.no_grad():
            xb = x
            if cfgn == 4:  # the rank's next batch of the corpus, synthesised on the device
                xb = synth_batch(B, n_samples, clip0=(state["batch"] * world + rank) * B, device=dev)
                state["batch"] += 1
            post, codes, _ = dec(enc(xb), vq=True)
            if cfgn == 3:
                state["wav"] = dec(post, vq=False)
            if world > 1:
                codes = all_gather_codes(codes)
            if cfgn == 4:  # int16 payload of the .npy files, every rank's clips
                c = codes if codes.ndim == 3 else codes.permute(1, 0, 2, 3).reshape(codes.shape[1], -1, codes.shape[3])
                state["host"] = batch_indices_to_numpy(c)
        return codes

    for _ in range(args.warmup):
        codes = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    state["batch"] = 0
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
        traffic, mutil, tsrc = pmc_traffic(kname)
        peak, mult, note = kernel_peak(kname)
        probe = mfma_probe_tflops(dev)
        practical = probe / mult if kname.startswith("conv1d_x6_kernel") else None
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "peak_note": note,
                "probe_bf16_tflops": round(probe, 1),
                "practical_peak": round(practical, 2) if practical else None,
                "practical_frac": round(achieved / practical, 4) if practical else None,
                "practical_note": "bc_mfma_probe: the dense-BF16 rate this device sustains on random register "
                                  "operands (its clock under MFMA load), / the kernel's MFMAs per FLOP pair",
                "mfma_tflops_executed": round(achieved * mult, 2),
                "traffic": round(traffic) if traffic else None, "traffic_source": tsrc,
                "pmc_mfma_util": round(mutil, 4) if mutil is not None else None,
                "algorithmic_bytes_per_launch": round(d["bytes_total"] / d["launches"]), "kernel": kname,
                "launches_per_step": d["launches"] // args.steps, "avg_launch_ms": round(avg_ms, 4),
                "algorithmic_gflop_per_launch": round(d["flops_total"] / d["launches"] / 1e9, 3),
                "all_python_conv_kernels_ms_per_step": round(conv_ms / args.steps, 2),
                "all_python_conv_tflops": round(sum(v["flops_total"] for v in summ.values()) / (conv_ms * 1e-3) / 1e12, 2),
                "kernels_top": kernel_table(summ, args.steps, probe)}

    cpu = None
    parity = None
    if rank == 0 and cfgn == 5:
        # index mismatch rate of the bf16 path against the fp32-accurate path on this batch
        got = (codes[0] if world > 1 else codes)[:, :B].cpu()
        _lib.set_precision("x6")
        with torch.no_grad():
            ref = dec(enc(x), vq=True)[1].cpu()
        _lib.set_precision(args.precision)
        parity = {"reference": "same batch through the fp32-accurate (x6) path", "frames": int(ref.numel()),
                  "index_mismatches": int((got != ref).sum()),
                  "mismatch_rate": round(float((got != ref).float().mean()), 5)}
    if rank == 0 and not args.no_cpu_baseline and cfgn == 6:
        cpu, wav_ref = cpu_decode_baseline(tok, sds, dk, args.cpu_clips)
        w = state["wav"][: args.cpu_clips].double().cpu()
        r = wav_ref.double()
        parity = {"clips_checked": args.cpu_clips, "samples": int(r.numel()),
                  "waveform_mse": float(((w - r) ** 2).mean()), "waveform_max_abs": float((w - r).abs().max()),
                  "note": "same codes through the CPU oracle's vq2emb + decoder"}
    if rank == 0 and not args.no_cpu_baseline and cfgn not in (5, 6):
        cpu, codes_ref, wav_ref = cpu_baseline(args.model, n_samples, sds, ek, dk, args.cpu_clips,
                                               roundtrip=cfgn == 3)
        got = codes[0] if world > 1 else codes
        if cfgn == 4:  # the last step's batch: recompute the first clip of rank 0's batch 0
            with torch.no_grad():
                got = dec(enc(x), vq=True)[1]
        got = got[:, : args.cpu_clips].cpu()
        parity = {"clips_checked": args.cpu_clips, "frames": int(got.numel()),
                  "index_mismatches": int((got != codes_ref).sum())}
        if cfgn == 3:
            w = state["wav"][: args.cpu_clips].double().cpu()
            r = wav_ref.double()
            parity["waveform_mse"] = float(((w - r) ** 2).mean())
            parity["waveform_max_abs"] = float((w - r).abs().max())
            parity["note"] = "waveforms compared end to end; equal codes make it the decoder's error alone"
    if rank == 0:
        dtype = {"fp32": "f32", "x6": "f32 (3xbf16-split MFMA, fp32 accumulate)",
                 "h3": "f32 (2xfp16 block-scaled split MFMA, fp32 accumulate)",
                 "bf16": "bf16 conv products, fp32 accumulate/storage (LSTM and VQ fp32-accurate)"}[args.precision]
        if cfgn == 4 and state["host"] is not None:
            assert state["host"].dtype == np.int16
        line = {
            "metric": METRIC_RT if cfgn == 3 else METRIC_DEC if cfgn == 6 else METRIC, "value": round(value, 2),
            "unit": "audio-sec/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic",
            "config": {"workload": f"config{cfgn}: batch={B} x {args.seconds:g} s {args.sample_rate // 1000} kHz "
                                   f"clips per GPU, {CONFIGS[cfgn]['work']}, BigCodec '{args.model}' model, "
                                   f"random weights",
                       "global_batch": B * world, "clip_samples": n_samples, "parallelism": f"dp{world}"},
            "roofline": roof, "cpu_baseline": cpu, "parity": parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
