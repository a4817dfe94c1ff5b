"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) into per-kernel HBM traffic per launch.

    python tools/pmc_summary.py gpurun_out/pmc profiles/r01_pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Per MI355X_MICROARCH.md §HBM, on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read; WRITE_SIZE is exact
for streaming stores.  A calibration on this code's own 4-B-per-lane transpose kernel (known bytes)
is recorded beside the result, and the traffic figure applies the guide's x2 read correction (an
upper bound for kernels whose reads are partly 4-B wide)."""
import collections
import csv
import json
import os
import sys


def load(path):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if name.startswith("void "):
            name = name[5:]
        name = name.split("(")[0].replace("bc::", "")
        out[name].append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    src, dst = sys.argv[1], sys.argv[2]
    fetch = load(os.path.join(src, "FETCH_SIZE", "run_counter_collection.csv"))
    write = load(os.path.join(src, "WRITE_SIZE", "run_counter_collection.csv"))
    res = {}
    for k in fetch:
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write.get(k, [0.0])) / max(1, len(write.get(k, [0.0])))
        res[k] = {"launches": len(fetch[k]), "fetch_bytes_raw": f, "write_bytes": w,
                  "traffic_bytes_corrected": 2.0 * f + w}
    out = {"note": "per-launch averages; traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 wide-read correction)",
           "kernels": res}
    calib = res.get("btc_to_ctb_kernel")
    if calib:
        out["calibration_btc_to_ctb"] = {"fetch_raw_over_known": None, "write_raw_bytes": calib["write_bytes"]}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: round(v["traffic_bytes_corrected"] / 1e9, 3) for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
