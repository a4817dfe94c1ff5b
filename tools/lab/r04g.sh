#!/bin/bash
# C = 96 ResidualUnit with the residual prefetched under phase 2: resunit parity tests, per-unit timing (encoder
# shapes, h3 / x6 / bf16), bench config 2.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -k "resunit or conv1d" > $O/gpu_tests.txt 2>&1
rc=$?; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; exit 1; }
for d in 1 3 9; do
  for p in h3 x6 bf16; do timeout -k 10 120 python tools/ru_bench.py --precision $p --C 96 --d $d --T 120000 --lazy >> $O/ru96.txt 2>&1 || exit 1; done
  timeout -k 10 120 python tools/ru_bench.py --precision x6 --C 48 --d $d --T 240000 --lazy >> $O/ru96.txt 2>&1 || exit 1
done
grep resunit $O/ru96.txt
timeout -k 10 500 python bench.py --no-cpu-baseline > $O/bench_config2.json 2> $O/bench_config2.err || { echo "bench failed $?"; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r04g/bench_config2.json").read().strip().splitlines()[-1])
r = d["roofline"]; x = d["x6"]
print(d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"], "x6", x["value"])
for row in r["kernels_top"]: print(row["kernel"], row["launches_per_step"], row["ms_per_step"], row["frac_mfma_spec"], row["frac_hbm"])
for row in x["roofline"]["kernels_top"]: print("x6", row["kernel"], row["launches_per_step"], row["ms_per_step"], row["frac_mfma_spec"])
PY
echo done
