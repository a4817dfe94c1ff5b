"""Benchmark of the BigCodec tokenization hot path on MI355X (BASELINE.json configs).

Default (what the driver runs) = BASELINE config 2: batch = 64 x 10 s @24 kHz clips per GPU, encode +
VQ (the extract_indices.py path: encoder -> decoder(vq=True) -> codes) of the `default` BigCodec
model in the reference's operand width (x6: every fp32 operand split exactly into three bf16 terms, 24 bits,
fp32 accumulation), synthetic white-noise clips already resident in HBM, random (counter-hash) weights.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5|6] [--precision h3|x6|fp32|bf16]

--gpus N > 1 starts N ranks itself (python -m torch.distributed.run as a child process, before this
process touches the GPU); under torchrun WORLD_SIZE must equal --gpus.  One process per GPU, RCCL.

--config 3: full encode -> VQ -> decode round trip (inference_full.py's model path), parity adds the
            decoder's waveform error against the CPU oracle decoding the same codes.
--config 4: extract_indices-style corpus streaming through extract.ShardedExtractor (the product's
            extract_sharded loop): every step is every rank's NEXT batch of a 100 k-clip corpus,
            synthesised on the device, encoded + quantised, its indices all-gathered (RCCL), and
            rank 0's sink receives every clip's int16 (F, Nq) .npy payload.
--config 5: batch = 32 x 30 s per GPU with bf16 conv products (precision 'bf16'); parity reports the
            index mismatch rate against the fp32-accurate path on the same batch.
--config 6: token -> audio decode (tokens.py service path).

A step = one batch per GPU through the path; for N > 1 each step ends with the RCCL all-gather of the
batch's index tensor (clip-sharded data parallelism, weak scaling).  Rank 0 prints one JSON line with
the whole-job throughput (audio-seconds per second, all GPUs), the roofline of the dominant kernel
(HIP-event timed inside the timed region), the CPU oracle baseline, the index parity of rank 0's batch
against the reference's full-size fixture (tests/golden/full_config2_default.npz: every mismatch with
its fp64 top-2 gap) and, for config 2, the same workload in the opt-in h3 arithmetic (22-bit operands:
narrower than the reference's fp32, reported as an extra leg only) beside the x6 headline.
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
    if kname.startswith(("lstm_seq2_x6_kernel", "pw_presplit_")) and len(targs) >= 2:  # <KS, P[, 1]>: P planes
        planes = targs[1]
    if kname.startswith(("pw_presplit_x6_kernel", "lstm_seq_x6_kernel")):
        planes = "3"
    if kname.startswith("pw_presplit_kernel"):  # the h3 pre-split GEMM
        planes = "2"
    if kname.startswith("conv1d_x6ra_kernel"):  # x6 (three bf16 planes) only
        planes = "3"
    if kname.startswith("resunit_w16_kernel") and targs:  # <P, SIN, B4>: x6 (3) or bf16 (1)
        planes = targs[0]
    if kname.startswith(("resunit_rr_kernel", "resunit_strip_kernel")):  # resunit_rr.hip: h3 (two fp16 planes) only
        planes = "2"
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


HBM_KERNELS = ("btc_to_ctb_kernel", "ctb_to_btc_add_kernel", "vq_fwd_kernel", "presplit_b_kernel", "presplit_b_x6_kernel")


def kernel_bound(name: str) -> str:
    """What bounds a kernel of the path: the layout transposes, the VQ (VALU argmin over 8192 codes
    per frame, z read once) and the B pre-split are HBM kernels; the persistent ResLSTM recurrence runs its x6
    MFMAs between per-step hand-offs of h_t (bound by that exchange: its MFMA fraction is reported, not reached);
    everything else is an MFMA GEMM."""
    if name.startswith(HBM_KERNELS):
        return "hbm"
    if name.startswith(("lstm_seq2_x6_kernel", "lstm_seq_x6_kernel")):
        return "mfma / h_t exchange"
    return "mfma"


def kernel_table(summ, steps, probe, n=12):
    """The n most time-consuming HIP-event-timed kernels of the timed steps: ms per step, algorithmic
    TFLOP/s against the kernel's MFMA ceiling (spec and probe-measured) and algorithmic GB/s against
    the 8 TB/s HBM peak.  The kernels' rows are the ones bench's roofline entry is drawn from.  Besides the
    Python-dispatched conv / ResidualUnit launches, the rows include the launches made inside the library's
    composite calls (the ResLSTM's transposes, projection and recurrence, the VQ: bc_launch_timer_*)."""
    rows = []
    for name, d in sorted(summ.items(), key=lambda kv: -kv[1]["ms_total"])[:n]:
        sec = d["ms_total"] * 1e-3
        tf = d["flops_total"] / sec / 1e12
        peak, mult, _ = kernel_peak(name)
        gbs = d["bytes_total"] / sec / 1e9
        bound = kernel_bound(name)
        rows.append({"kernel": name, "bound": bound, "launches_per_step": d["launches"] // steps,
                     "ms_per_step": round(d["ms_total"] / steps, 3), "tflops": round(tf, 1),
                     "frac_mfma_spec": round(tf / peak, 3) if bound != "hbm" else None,
                     "frac_mfma_probe": round(tf * mult / probe, 3) if name.startswith(("conv1d_x6", "resunit_", "pw_presplit", "lstm_seq")) else None,
                     "gbs": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 3)})
    return rows


def roofline(summ, steps, probe):
    """The `roofline` object of the JSON line: the dominant HIP-event-timed kernel (largest total time over the
    timed steps), its algorithmic TFLOP/s at its average launch duration against its MFMA ceiling (spec and
    probe-measured), the newest committed PMC traffic / MFMA utilisation of that kernel, and kernels_top."""
    kname, d = max(summ.items(), key=lambda kv: kv[1]["ms_total"])
    avg_ms = d["ms_total"] / d["launches"]
    achieved = d["flops_total"] / d["launches"] / (avg_ms * 1e-3) / 1e12
    conv = {k: v for k, v in summ.items() if k.startswith(("conv1d_", "resunit_"))}
    conv_ms = sum(v["ms_total"] for v in conv.values())
    traffic, mutil, tsrc = pmc_traffic(kname)
    peak, mult, note = kernel_peak(kname)
    practical = probe / mult if kname.startswith(("conv1d_x6_kernel", "conv1d_x6ra_kernel")) else None
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
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
            "launches_per_step": d["launches"] // steps, "avg_launch_ms": round(avg_ms, 4),
            "algorithmic_gflop_per_launch": round(d["flops_total"] / d["launches"] / 1e9, 3),
            "all_python_conv_kernels_ms_per_step": round(conv_ms / steps, 2),
            "all_python_conv_tflops": round(sum(v["flops_total"] for v in conv.values()) / (conv_ms * 1e-3) / 1e12, 2),
            "all_timed_kernels_ms_per_step": round(sum(v["ms_total"] for v in summ.values()) / steps, 2),
            "kernels_top": kernel_table(summ, steps, probe)}


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
    p.add_argument("--cpu-clips", type=int, default=4, help="clips in the CPU-baseline B=1 sample (about 3 s each)")
    p.add_argument("--cpu-batches", default="4,16", help="batch sizes of the extra CPU-baseline calls ('' = none)")
    p.add_argument("--no-h3", action="store_true", help="skip the 22-bit h3 leg beside the x6 headline")
    p.add_argument("--h3-steps", type=int, default=None, help="timed steps of the h3 leg (default: --steps)")
    p.add_argument("--corpus", type=int, default=100_000, help="config 4: clips in the synthetic corpus")
    p.add_argument("--precision", choices=["fp32", "x6", "bf16", "h3"], default=None,
                   help="conv GEMM arithmetic (default: the config's, else BIGCODEC_PRECISION or x6)")
    a = p.parse_args()
    c = CONFIGS[a.config]
    a.batch = a.batch or c["batch"]
    a.seconds = a.seconds or c["seconds"]
    a.precision = a.precision or c["precision"]
    a.h3_steps = a.h3_steps or a.steps  # the h3 leg is timed over as many steps as the headline
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


def pmc_traffic(kernel: str, running: str | None = None, profiles: str | None = None):
    """(HBM bytes per launch, MFMA utilisation, source file) of `kernel` from the newest committed PMC
    summary (tools/gpu_pmc.sh -> tools/pmc_summary.py -> profiles/*pmc_traffic.json) that was taken on a library
    with the RUNNING library's source digest (bc_build_digest), or Nones: a profile of other kernel code is never
    reported as this run's traffic."""
    import glob

    from audiotokenization_amd import _lib

    if running is None:
        running = _lib.load().bc_build_digest().decode()
    files = sorted(glob.glob(os.path.join(profiles or os.path.join(REPO, "profiles"), "*pmc_traffic.json")))
    for f in reversed(files):
        try:
            j = json.load(open(f))
            d = j.get("kernels", {}).get(kernel)
        except (OSError, ValueError, AttributeError):  # a malformed summary must not take the bench down
            continue
        if d and "traffic_bytes_corrected" in d and j.get("lib_digest") == running:
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


def cpu_info():
    """(threads to use, description): the physical cores this process may run on — the affinity set
    mapped to (package, core) pairs via /proc/cpuinfo, capped by a cgroup CPU quota (cpu.max) when one
    is set — and the CPU model name."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    model, cores, cur = None, set(), {}
    try:
        for line in open("/proc/cpuinfo").read().split("\n") + [""]:
            if not line.strip():
                if cur.get("processor") is not None and int(cur["processor"]) in aff:
                    cores.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                cur = {}
                continue
            k, _, v = line.partition(":")
            cur[k.strip()] = v.strip()
            if k.strip() == "model name" and model is None:
                model = v.strip()
    except OSError:
        pass
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(p)))
    except (OSError, ValueError):
        pass
    phys = len(cores) or len(aff)
    threads = max(1, min(phys, quota or phys))
    desc = (f"{model or 'unknown CPU'}; {len(aff)} logical CPUs in affinity = {phys} physical cores"
            + (f", cgroup quota {quota} CPUs" if quota else ", no cgroup CPU quota") + f" -> {threads} threads")
    return threads, desc


def cpu_baseline(name, n_samples, sds, ek, dk, n_clips, roundtrip=False, batches=(1, 4, 16)):
    """The CPU oracle (torch CPU restatement, bit-identical to the reference in the development
    container) timed on this host with every physical core available to the process:
    encode + VQ (+ decode for the round trip), B = 1 per clip (extract_indices.py:397) over `n_clips`
    clips, plus one call of each batch size in `batches` > 1 (best of B in {1, 4, 16}), warm.
    Returns (baseline dict, codes (Nq, n_clips, F), embeddings, waveforms or None)."""
    import torch

    from audiotokenization_amd import synth
    from oracle import bigcodec_oracle as O

    threads, desc = cpu_info()
    torch.set_num_threads(threads)
    nb = max([n_clips] + [b for b in batches if not roundtrip])
    x = torch.from_numpy(synth.synth_clips(nb, n_samples, clip0=0)).unsqueeze(1)
    codes, embs, wavs = [], [], []
    with torch.no_grad():
        O.encode_indices(x[:1, :, : n_samples // 10], sds[0], sds[1], ek, dk)  # warm-up (short)
        t0 = time.perf_counter()
        for i in range(n_clips):
            c, emb = O.encode_indices(x[i:i + 1], sds[0], sds[1], ek, dk)
            codes.append(c)
            embs.append(emb)
            if roundtrip:
                zq, _, _ = O.rvq_forward(emb, sds[1], "quantizer.", dk.get("vq_num_quantizers", 1))
                wavs.append(O.decoder_forward(zq, sds[1], dk))
        dt = time.perf_counter() - t0
        rates = {"B=1": n_clips * n_samples / 24000.0 / dt}
        total = dt
        if not roundtrip:
            for b in batches:
                if b <= 1:
                    continue
                t0 = time.perf_counter()
                O.encode_indices(x[:b], sds[0], sds[1], ek, dk)
                tb = time.perf_counter() - t0
                total += tb
                rates[f"B={b}"] = b * n_samples / 24000.0 / tb
    what = "encode+VQ+decode" if roundtrip else "encode+VQ"
    best = max(rates, key=rates.get)
    return (dict(value=rates[best], unit="audio-sec/s", cores=threads, kind="port", rates=rates, cpu=desc,
                 b1_value=rates["B=1"],
                 sample=f"{n_clips} clip(s) x {n_samples / 24000:.0f} s @24 kHz at B=1"
                        + "".join(f", 1 call at {k}" for k in rates if k != "B=1")
                        + f"; {name} model, {what}, torch CPU oracle (bit-identical to the reference in the "
                          f"development container), best = {best} (B=1 is extract_indices.py:397), {total:.1f} s"),
            torch.cat(codes, dim=1), torch.cat(embs, dim=0), torch.cat(wavs, dim=0) if roundtrip else None)


def vq_gaps(emb, dec_sd):
    """fp64 top-2 distance gap of every frame of the oracle's latent (the certificate of a flip)."""
    import torch

    from oracle import bigcodec_oracle as O

    z_e = O.fvq_forward(emb, dec_sd, "quantizer.layers.0.", return_ze=True)[3]
    b, d, t = z_e.shape
    e = z_e.permute(0, 2, 1).reshape(-1, d).double()
    e = e / e.norm(dim=1, keepdim=True).clamp_min(1e-12)
    c = dec_sd["quantizer.layers.0._codebook.weight"].double()
    c = c / c.norm(dim=1, keepdim=True).clamp_min(1e-12)
    dist = (e * e).sum(1, keepdim=True) - 2 * e @ c.t() + (c * c).sum(1)[None]
    v, _ = torch.topk(dist, 2, dim=1, largest=False)
    return (v[:, 1] - v[:, 0]).reshape(b, t).numpy()


GAP_TOL = 1e-6  # a flip is certified only at a frame whose fp64 top-2 gap is below this (tests/helpers.py)


def mismatch_report(got, want, gap, reference):
    """Every index mismatch with its certified fp64 top-2 gap."""
    import numpy as np

    got = np.asarray(got).reshape(want.shape)
    bad = np.argwhere(got != want)
    items = [{"clip": int(b), "frame": int(f), "got": int(got[b, f]), "want": int(want[b, f]),
              "gap": float(gap[b, f])} for b, f in bad[:64]]
    worst = max((float(gap[b, f]) for b, f in bad), default=0.0)
    return {"reference": reference, "frames": int(want.size), "index_mismatches": int(len(bad)),
            "mismatches": items, "worst_gap": worst, "gap_tol": GAP_TOL, "all_certified": worst <= GAP_TOL,
            "min_gap_all_frames": float(np.min(gap))}


def golden_parity(codes, model, n_samples, B):
    """Rank 0's batch (clips 0..B-1) against tests/golden/full_config2_default.npz: the REFERENCE's
    indices for clips 0..63 x 240 000 samples of the default model (tools/make_golden_full.py), every
    mismatch listed with its fp64 top-2 gap.  None when the workload is not that fixture's."""
    import numpy as np

    path = os.path.join(REPO, "tests", "golden", "full_config2_default.npz")
    if model != "default" or n_samples != 240_000 or not os.path.exists(path):
        return None
    g = np.load(path)
    n = min(B, g["codes"].shape[0])
    got = codes[0, :n].cpu().numpy()
    return mismatch_report(got, g["codes"][:n].astype(np.int64), g["gap"][:n],
                           f"reference CPU path (tests/golden/full_config2_default.npz, clips 0-{n - 1})")


def cpu_decode_baseline(codes, sds, dk, n_clips):
    """The CPU oracle's token -> audio decode (vq2emb -> transpose -> decoder) on this host, B = 1 per
    clip, warm.  Returns (baseline dict, waveforms)."""
    import numpy as np
    import torch

    from oracle import bigcodec_oracle as O

    threads, desc = cpu_info()
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
    return (dict(value=audio_s / dt, unit="audio-sec/s", cores=threads, kind="port", cpu=desc,
                 sample=f"{n_clips} clip(s) x {codes.shape[1]} frames, token -> audio decode, B=1, torch CPU "
                        f"oracle, {dt:.1f} s"),
            torch.cat(wavs, dim=0))


def launch_ranks(args):
    """--gpus N > 1 without a torch.distributed environment: start N ranks as CHILD processes
    (python -m torch.distributed.run ...) before this process touches the GPU, and exit with their
    code.  Under a launcher, WORLD_SIZE must equal --gpus."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={env_world} disagrees with --gpus {args.gpus}")
        return
    if args.gpus <= 1:
        return
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    sys.exit(subprocess.call(cmd, env=env))


def main():
    args = parse()
    launch_ranks(args)
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
    from audiotokenization_amd.extract import ShardedExtractor, all_gather_codes, synth_batch

    _lib.load()
    if args.precision:
        _lib.set_precision(args.precision)
    args.precision = _lib.precision_name()
    n_samples = int(round(args.seconds * args.sample_rate))
    enc, dec, sds, ek, dk = build_model(args.model, dev)
    B = args.batch
    cfgn = args.config
    x = synth_batch(B, n_samples, clip0=rank * B, device=dev)  # resident in HBM before timing
    state = {"wav": None, "host": 0}
    tok = None
    if cfgn == 6:  # synthetic codes of the clips' frame count, uniform over the codebook, seeded per rank
        n_frames = n_samples // int(dec.hop_length)
        g = torch.Generator().manual_seed(1234 + rank)
        tok = torch.randint(0, dec.quantizer.layers[0].codebook_size, (B, n_frames, 1), generator=g)
        tok_dev = tok.to(dev)
    extractor = None
    if cfgn == 4:  # the 100 k-clip corpus, clip-sharded; every step is the next batch of every rank
        def sink(cid, arr):  # rank 0 receives every clip's (F, Nq) int16 .npy payload (file writes excluded)
            state["host"] += 1

        extractor = ShardedExtractor(lambda xb: dec(enc(xb), vq=True)[1], args.corpus, n_samples, B, rank, world,
                                     dev, sink=sink)
        state["bi"] = 0

    def step():
        if cfgn == 6:
            with torch.no_grad():
                state["wav"] = dec.tokens_to_audio(tok_dev)
            return None
        with torch.no_grad():
            if cfgn == 4:  # extract_sharded's loop body: synthesise, encode + VQ, gather, int16 host copy
                codes = extractor.step(state["bi"])
                state["bi"] += 1
                return codes
            post, codes, _ = dec(enc(x), vq=True)
            if cfgn == 3:
                state["wav"] = dec(post, vq=False)
            if world > 1:
                codes = all_gather_codes(codes)
        return codes

    def timed(n_steps, timer=None):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        _lib.set_timer(timer)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(n_steps):
            codes = step()
        if extractor is not None:
            extractor.flush()  # rank 0's sink has received every timed batch (its writer thread runs behind)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        _lib.set_timer(None)
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, codes

    for _ in range(args.warmup):
        codes = step()
    timer = None if args.no_kernel_timer else _lib.KernelTimer()
    elapsed, codes = timed(args.steps, timer)
    if cfgn == 4:
        assert extractor.stats.errors == 0 and extractor.stats.job_errors == 0, extractor.stats

    audio_s = world * B * n_samples / args.sample_rate * args.steps
    value = audio_s / elapsed
    probe = None
    roof = None
    if timer is not None:
        probe = mfma_probe_tflops(dev)
        roof = roofline(timer.summary(), args.steps, probe)

    # rank 0's own batch codes (Nq, B, F) of the last timed step, for parity
    mine = None
    if cfgn in (2, 3):
        mine = (codes[0] if world > 1 else codes)[:, :B]
    elif cfgn == 4:
        with torch.no_grad():
            mine = dec(enc(x), vq=True)[1]  # rank 0's batch 0 = clips 0..B-1 (block partition at rank 0)

    # opt-in h3 leg (22-bit block-scaled operands, narrower than the reference's fp32) beside the x6 headline:
    # same workload, own timing; reported, never the headline
    h3 = None
    if cfgn == 2 and args.precision == "x6" and not args.no_h3:
        _lib.set_precision("h3")
        for _ in range(1):
            step()
        timer3 = None if args.no_kernel_timer else _lib.KernelTimer()
        el3, codes3 = timed(args.h3_steps, timer3)
        _lib.set_precision(args.precision)
        v3 = world * B * n_samples / args.sample_rate * args.h3_steps / el3
        h3 = {"precision": "h3 (opt-in, NOT the reference's width): fp32 operands block-scaled and split into 2 fp16 "
                           "terms (22-bit operands), 3 fp16 MFMAs per product, fp32 accumulate",
              "value": round(v3, 2), "ms_per_step": round(el3 / args.h3_steps * 1e3, 2), "steps": args.h3_steps,
              "roofline": roofline(timer3.summary(), args.h3_steps, probe) if timer3 is not None else None}
        if rank == 0:
            h3["parity"] = golden_parity((codes3[0] if world > 1 else codes3)[:, :B], args.model, n_samples, B)

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
    if rank == 0 and cfgn in (2, 3, 4):
        parity = {}
        full = golden_parity(mine, args.model, n_samples, B)
        if full is not None:
            parity["vs_reference_fixture"] = full
        if not args.no_cpu_baseline:
            batches = tuple(int(b) for b in args.cpu_batches.split(",")) if args.cpu_batches else ()
            cpu, codes_ref, emb_ref, wav_ref = cpu_baseline(args.model, n_samples, sds, ek, dk, args.cpu_clips,
                                                            roundtrip=cfgn == 3, batches=batches)
            n = args.cpu_clips
            parity["vs_cpu_oracle"] = mismatch_report(mine[0, :n].cpu().numpy(), codes_ref[0].numpy(),
                                                      vq_gaps(emb_ref, sds[1]),
                                                      f"CPU oracle run here on clips 0-{n - 1}")
            if cfgn == 3:
                w = state["wav"][:n].double().cpu()
                r = wav_ref.double()
                parity["waveform_mse"] = float(((w - r) ** 2).mean())
                parity["waveform_max_abs"] = float((w - r).abs().max())
                parity["note"] = "waveforms compared end to end; equal codes make it the decoder's error alone"
    if rank == 0:
        prec = {"fp32": ("f32", "native fp32 MFMA (v_mfma_f32_16x16x4f32)"),
                "x6": ("f32-emulated (x6: 3xbf16, 24-bit operands)",
                       "fp32-class: operands split exactly into 3 bf16 terms (24-bit), 6 bf16 MFMAs per "
                       "product, fp32 accumulate"),
                "h3": ("f32-emulated (h3: 2xfp16, 22-bit operands, narrower than fp32)",
                       "fp32-class: operands block-scaled and split into 2 fp16 terms (22-bit), 3 fp16 "
                       "MFMAs per product (lo x lo dropped, < 2^-22 relative), fp32 accumulate"),
                "bf16": ("bf16", "bf16 conv products (one bf16 MFMA per product), fp32 accumulate and storage; "
                                 "ResLSTM on h3 (fp32-class, 22-bit operands), VQ fp32 (IEEE op order)")}[args.precision]
        line = {
            "metric": METRIC_RT if cfgn == 3 else METRIC_DEC if cfgn == 6 else METRIC, "value": round(value, 2),
            "unit": "audio-sec/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": prec[0],
            "precision": {"mode": args.precision, "arithmetic": prec[1]}, "data": "synthetic",
            "config": {"workload": f"config{cfgn}: batch={B} x {args.seconds:g} s {args.sample_rate // 1000} kHz "
                                   f"clips per GPU, {CONFIGS[cfgn]['work']}, BigCodec '{args.model}' model, "
                                   f"random weights" + (f", corpus of {args.corpus} clips" if cfgn == 4 else ""),
                       "global_batch": B * world, "clip_samples": n_samples, "parallelism": f"dp{world}"},
            "roofline": roof, "cpu_baseline": cpu, "parity": parity, "h3": h3,
            # the RUNNING library's source digest (bc_build_digest): tools/pmc_summary.py stamps a PMC summary with the
            # digest the profiled bench printed here, not with whatever library the package holds when it is written
            "lib_digest": _lib.load().bc_build_digest().decode(),
        }
        if cfgn == 4:
            line["extract"] = {"batches_per_rank": args.steps, "clips_sunk_rank0": state["host"],
                               "errors": extractor.stats.job_errors}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
