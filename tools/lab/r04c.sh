#!/bin/bash
# Round 4 pass 2: the remaining GPU tests from the streaming module on, then the x6 tile sweep, bench config 2
# (h3 + x6 leg with its roofline) and config 5.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_streaming.py tests/test_gpu_extract.py tests/test_extract_cli.py tests/test_gpu_full_size.py tests/test_gpu_configs.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -3 $O/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; exit 1; }
grep -E "config (4|5)|stream decode" $O/gpu_tests.txt | grep -v "print\|f\"" | head -20
rm -f gpurun_out/x6_sweep.log
bash tools/x6_table_sweep.sh || exit 1
cp gpurun_out/x6_sweep.log $O/
timeout -k 10 500 python bench.py > $O/bench_config2.json 2> $O/bench_config2.err || { echo "bench failed $?"; tail -5 $O/bench_config2.err; exit 1; }
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > $O/bench_config5.json 2> $O/bench_config5.err || { echo "config 5 failed $?"; exit 1; }
python - <<'PY'
import json
for c in (2, 5):
    d = json.loads(open(f"gpurun_out/r04c/bench_config{c}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(c, d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"])
    if d.get("x6"):
        x = d["x6"]; rr = x["roofline"]
        print("x6", x["value"], x["ms_per_step"], rr["kernel"], rr["avg_launch_ms"], rr["frac"], x["parity"]["index_mismatches"])
PY
echo done
