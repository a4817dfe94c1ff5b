#!/bin/bash
# Round 3: the one-launch ResidualUnits at the config-2 shapes (h3, snake on load, as the encoder flow runs them)
# plus their parity tests.  One GPU process per line; the first failure ends the script.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03_ru_probe.txt; : > $o
run() { timeout -k 10 120 python tools/ru_bench.py --precision h3 --iters 5 --lazy "$@" >> $o 2>&1 || { echo "failed: $*" >> $o; exit 1; }; }
for d in 1 3 9; do run --C 48 --d $d --T 240000; done
for d in 1 3 9; do run --C 96 --d $d --T 120000; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "resunit" -x -q --timeout 120 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
echo done >> $o
