#!/bin/bash
# Round 4: the decoder's kernel mix (config 6, token -> audio) under rocprofv3 kernel stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c6 -o run -- \
  python3 bench.py --config 6 --no-cpu-baseline --no-x6 --steps 3 --warmup 1 > $O/c6.log 2>&1 || { echo "c6 failed $?"; tail $O/c6.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04o/c6/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:8.3f} ms  {r['Name'][:110]}")
PY
