#!/bin/bash
# Round 4 pass 3 (x6 table): every -m gpu test, bench config 2 (h3 + x6 leg), rocprofv3 kernel stats of the h3 and
# the x6 bench, PMC passes (FETCH_SIZE / WRITE_SIZE / MFMA) of both.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; exit 1; }
timeout -k 10 500 python bench.py > $O/bench_config2.json 2> $O/bench_config2.err || { echo "bench failed $?"; tail -5 $O/bench_config2.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_h3 -o run -- \
  python3 bench.py --no-cpu-baseline --no-x6 > $O/stats_h3.log 2>&1 || { echo "h3 stats failed $?"; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_x6 -o run -- \
  python3 bench.py --no-cpu-baseline --precision x6 > $O/stats_x6.log 2>&1 || { echo "x6 stats failed $?"; exit 1; }
PMC_DIR=$O/pmc_h3 PMC_TIMEOUT=300 bash tools/gpu_pmc.sh || { echo "pmc h3 failed $?"; exit 1; }
PMC_DIR=$O/pmc_x6 PMC_TIMEOUT=300 BENCH_ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timer --precision x6" bash tools/gpu_pmc.sh || { echo "pmc x6 failed $?"; exit 1; }
python tools/pmc_summary.py $O/pmc_h3 $O/pmc_h3.json > $O/pmc_h3.txt
python tools/pmc_summary.py $O/pmc_x6 $O/pmc_x6.json > $O/pmc_x6.txt
rm -rf $O/pmc_h3/*/ $O/pmc_x6/*/ 2>/dev/null
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r04d/bench_config2.json").read().strip().splitlines()[-1])
r = d["roofline"]; x = d["x6"]; rr = x["roofline"]
print(d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"])
print("x6", x["value"], x["ms_per_step"], rr["kernel"], rr["avg_launch_ms"], rr["frac"], x["parity"]["index_mismatches"])
PY

# one-launch ResidualUnit: 8-wave 96 x 128 (323) vs 16-wave 96 x 256 (325) at C = 96, strip vs 16-wave 48 x 512 (326)
# at C = 48, h3, snake on load (as the encoder runs them), encoder shapes
for d in 1 3 9; do
  for c in 323 325; do timeout -k 10 120 python tools/ru_bench.py --C 96 --d $d --T 120000 --lazy --cfg $c >> $O/ru_ab.txt 2>&1 || exit 1; done
  for c in 311 326; do timeout -k 10 120 python tools/ru_bench.py --C 48 --d $d --T 240000 --lazy --cfg $c >> $O/ru_ab.txt 2>&1 || exit 1; done
done
for d in 1 9; do
  for c in 323 325; do BC_RU_TPS=4 timeout -k 10 120 python tools/ru_bench.py --C 96 --d $d --T 120000 --lazy --cfg $c >> $O/ru_ab.txt 2>&1 || exit 1; done
done
grep resunit $O/ru_ab.txt
echo done
