"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) into per-kernel HBM traffic and MFMA
utilisation per launch.

    python tools/pmc_summary.py gpurun_out/pmc profiles/r01_pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Per MI355X_MICROARCH.md §HBM, on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read; WRITE_SIZE is exact
for streaming stores.  traffic = 2 * FETCH_SIZE + WRITE_SIZE (the guide's x2 read correction; an
upper bound for kernels whose reads are partly 4-B wide).

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the busy
cycles of the matrix pipes (16 per v_mfma_f32_16x16x32_bf16, checked against the algorithmic MFMA
count of the C = 384 k=7 conv) over the SIMD-cycles the dispatch was resident, at the clock it ran."""
import collections
import csv
import json
import os
import sys

N_XCD, N_SIMD = 8, 1024


def load(path, counter=None):
    out = collections.defaultdict(list)
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        if counter and r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if name.startswith("void "):
            name = name[5:]
        name = name.split("(")[0].replace("bc::", "")
        out[name].append(float(r["Counter_Value"]))
    return out


def mean(v):
    return sum(v) / len(v) if v else 0.0


def profiled_digest(src):
    """The library digest the profiled bench itself printed (its JSON line's lib_digest) in every pass log of
    tools/gpu_pmc.sh, or None when a log lacks it or the passes ran different libraries (reading the
    package's .so here would stamp an A/B build's or a rebuilt library's counters with the wrong digest)."""
    digs = set()
    for pass_ in ("FETCH_SIZE", "WRITE_SIZE", "MFMA"):
        path = os.path.join(src, pass_ + ".log")
        if not os.path.exists(path):
            continue
        dig = None
        for line in open(path, errors="replace"):
            line = line.strip()
            if line.startswith("{") and '"lib_digest"' in line:
                try:
                    dig = json.loads(line).get("lib_digest")
                except ValueError:
                    pass
        digs.add(dig)
    if len(digs) != 1 or None in digs:
        print(f"pmc_summary: pass logs name digests {sorted(map(str, digs))}: lib_digest left null", file=sys.stderr)
        return None
    return digs.pop()


def main():
    src, dst = sys.argv[1], sys.argv[2]
    fetch = load(os.path.join(src, "FETCH_SIZE", "run_counter_collection.csv"))
    write = load(os.path.join(src, "WRITE_SIZE", "run_counter_collection.csv"))
    mp = os.path.join(src, "MFMA", "run_counter_collection.csv")
    busy = load(mp, "SQ_VALU_MFMA_BUSY_CYCLES")
    gui = load(mp, "GRBM_GUI_ACTIVE")
    res = {}
    for k in fetch:
        f = mean(fetch[k]) * 1024.0
        w = mean(write.get(k, [])) * 1024.0
        d = {"launches": len(fetch[k]), "fetch_bytes_raw": f, "write_bytes": w,
             "traffic_bytes_corrected": 2.0 * f + w}
        if busy.get(k) and gui.get(k):
            util = [b / (g / N_XCD * N_SIMD) for b, g in zip(busy[k], gui[k]) if g > 0]
            d["mfma_util"] = mean(util)
            d["mfma_busy_cycles"] = mean(busy[k])
        res[k] = d
    out = {"lib_digest": profiled_digest(src),  # bench.py reports this traffic only on that library
           "note": "per-launch averages; traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 wide-read correction); "
                   "mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)",
           "kernels": res}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes_corrected"] * kv[1]["launches"]):
        print(f"{k:60s} x{v['launches']:3d}  traffic {v['traffic_bytes_corrected'] / 1e9:8.3f} GB/launch"
              + (f"  mfma_util {v['mfma_util']:.3f}" if "mfma_util" in v else ""))


if __name__ == "__main__":
    main()
