#!/bin/bash
# Round 4: kernel mix of a narrow decode / encode stream push after the narrow-launch tiles.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
for m in dec enc; do
  if [ $m = dec ]; then A="--decode --B 16 --chunk 1000"; else A="--B 16 --chunk 1200"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o run -- \
    python3 tools/stream_bench.py $A --reps 1 > $O/$m.log 2>&1 || { echo "$m failed $?"; tail $O/$m.log; exit 1; }
done
python3 - <<'PY'
import csv
for m, pushes in (("dec", 480), ("enc", 400)):
    rows = list(csv.DictReader(open(f"gpurun_out/r04w/{m}/run_kernel_stats.csv")))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{m}: kernels {tot/1e6:.1f} ms = {tot/1e3/pushes:.0f} us per push")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
        print(f"  {float(r['TotalDurationNs'])/1e3/pushes:7.1f} us/push {int(r['Calls'])/pushes:5.1f}/push {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:80]}")
PY
