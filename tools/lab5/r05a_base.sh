#!/bin/bash
# round 5 baseline: the x6-headline bench line (h3 leg beside it), rocprof stats of the x6 bench, x6 layer profile
set -u
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-clips 1 --cpu-batches "" > $O/bench.json 2> $O/bench.err || { echo "bench failed $?"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python tools/layer_profile.py --precision x6 > $O/layers_x6.txt 2>&1 || { echo "layers failed $?"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_x6 -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-h3 > $O/stats_x6.log 2>&1 || { echo "x6 stats failed $?"; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05a/bench.json").read().strip().splitlines()[-1])
r = d["roofline"]; x = d["h3"]; rr = x["roofline"]
print("x6 headline", d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"], d["parity"]["vs_reference_fixture"]["index_mismatches"])
print("h3 leg", x["value"], x["ms_per_step"], rr["kernel"], rr["avg_launch_ms"], rr["frac"], x["parity"]["index_mismatches"])
for k in r["kernels_top"]: print(k)
PY
echo done
