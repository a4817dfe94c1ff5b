#!/bin/bash
# Round 3 iteration check: kernel + model GPU tests, C = 48 unit timing, config-2 bench.  First failure ends it.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03_check2.txt; : > $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
for d in 1 3 9; do
  timeout -k 10 120 python tools/ru_bench.py --precision h3 --iters 5 --lazy --C 48 --d $d --T 240000 >> $o 2>&1 || { echo "bench failed" >> $o; exit 1; }
done
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-x6 > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err || { echo "bench.py failed $?" >> $o; exit 1; }
echo done >> $o
