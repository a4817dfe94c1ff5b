#!/bin/bash
# Round 4: what a narrow stream push spends now (rocprof), and the pointwise convs' tiles at narrow shapes.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
run() { timeout -k 10 240 python tools/conv_bench.py --precision h3 --cfg all --iters 20 "$@" >> $O/sweep.txt 2>&1 || { echo "failed $? on $*"; tail -3 $O/sweep.txt; exit 1; }; }
run --cin 768 --cout 768 --k 1 --T 25 --B 16 --res --dual
run --cin 384 --cout 384 --k 1 --T 125 --B 16 --res --dual
run --cin 768 --cout 768 --k 1 --T 120 --B 64 --res --dual
run --cin 1536 --cout 1536 --k 1 --T 24 --B 64 --res
grep "best cfg" $O/sweep.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec -o run -- \
  python3 tools/stream_bench.py --decode --B 16 --chunk 1000 --reps 1 > $O/dec.log 2>&1 || { echo "dec failed $?"; tail $O/dec.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04u/dec/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"decode stream kernels total {tot/1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f"  {float(r['TotalDurationNs'])/1e6:8.2f} ms {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.1f} us {r['Name'][:90]}")
PY
