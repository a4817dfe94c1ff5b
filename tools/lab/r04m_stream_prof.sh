#!/bin/bash
# Round 4: where a streaming push goes -- kernel time vs wall time (rocprofv3 kernel stats of the stream benches).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o run -- \
  python3 tools/stream_bench.py --decode --B 16 --chunk 1000 --reps 1 > $O/dec.log 2>&1 || { echo "dec failed $?"; tail $O/dec.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/enc -o run -- \
  python3 tools/stream_bench.py --chunk 4800 --reps 1 > $O/enc.log 2>&1 || { echo "enc failed $?"; tail $O/enc.log; exit 1; }
grep stream $O/dec.log $O/enc.log
python3 - <<'PY'
import csv, glob
for tag in ("dec", "enc"):
    f = glob.glob(f"gpurun_out/r04m/{tag}/**/run_kernel_stats.csv", recursive=True) + glob.glob(f"gpurun_out/r04m/{tag}/run_kernel_stats.csv")
    rows = list(csv.DictReader(open(f[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    calls = sum(int(r["Calls"]) for r in rows)
    print(tag, f"kernels total {tot/1e6:.1f} ms over {calls} launches")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
        print(f"  {float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us {r['Name'][:90]}")
PY
