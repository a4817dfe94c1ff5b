#!/bin/bash
# End-of-round regression, part A: smoke, every -m gpu test, the default bench line (what the driver runs).
set -u
mkdir -p gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.txt 2>&1 || { echo "smoke failed $?"; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.txt 2>&1 || { echo "gpu tests failed $?"; tail -30 gpurun_out/final/gpu_tests.txt; exit 1; }
timeout -k 10 500 python bench.py > gpurun_out/final/bench_config2.json 2> gpurun_out/final/bench_config2.err || { echo "bench failed $?"; exit 1; }
tail -1 gpurun_out/final/gpu_tests.txt
echo done
