#!/bin/bash
# End-of-round regression on ONE box (round 4): smoke, every -m gpu test, the default bench line (h3 headline + x6 leg,
# CPU baseline), rocprofv3 kernel stats of the h3 and x6 benches, configs 3-6, PMC passes of both benches.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed $?"; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed $?"; grep -E "^E |FAILED" $O/gpu_tests.txt | head; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 500 python bench.py > $O/bench_config2.json 2> $O/bench_config2.err || { echo "bench failed $?"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_h3 -o run -- \
  python3 bench.py --no-cpu-baseline --no-x6 > $O/stats_h3.log 2>&1 || { echo "h3 stats failed $?"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_x6 -o run -- \
  python3 bench.py --no-cpu-baseline --precision x6 > $O/stats_x6.log 2>&1 || { echo "x6 stats failed $?"; exit 1; }
for c in 3 4 5 6; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-x6 > $O/bench_config$c.json 2> $O/bench_config$c.err || { echo "config $c failed $?"; exit 1; }
done
PMC_DIR=$O/pmc_h3 PMC_TIMEOUT=300 bash tools/gpu_pmc.sh || { echo "pmc h3 failed $?"; exit 1; }
PMC_DIR=$O/pmc_x6 PMC_TIMEOUT=300 BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timer --precision x6" bash tools/gpu_pmc.sh || { echo "pmc x6 failed $?"; exit 1; }
python tools/pmc_summary.py $O/pmc_h3 $O/pmc_h3.json > $O/pmc_h3.txt
python tools/pmc_summary.py $O/pmc_x6 $O/pmc_x6.json > $O/pmc_x6.txt
rm -rf $O/pmc_h3/*/ $O/pmc_x6/*/ 2>/dev/null
python - <<'PY'
import json
d = json.loads(open("gpurun_out/final/bench_config2.json").read().strip().splitlines()[-1])
r = d["roofline"]; x = d["x6"]; rr = x["roofline"]
print("config2", d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"],
      d["parity"]["vs_reference_fixture"]["index_mismatches"], "cpu", d["cpu_baseline"]["value"])
print("x6", x["value"], x["ms_per_step"], rr["kernel"], rr["avg_launch_ms"], rr["frac"], x["parity"]["index_mismatches"])
for c in (3, 4, 5, 6):
    e = json.loads(open(f"gpurun_out/final/bench_config{c}.json").read().strip().splitlines()[-1])
    print(f"config{c}", e["value"], e["ms_per_step"], e["roofline"]["kernel"], e["roofline"]["frac"])
PY
echo done
