#!/bin/bash
# Round 3: the streaming C = 48 ResidualUnit: parity tests, per-launch timing (strip vs resunit_rr), config 2 bench.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03_strip.txt; : > $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "resunit" -x -q -s --timeout 120 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
for d in 1 3 9; do
  timeout -k 10 120 python tools/ru_bench.py --precision h3 --iters 5 --lazy --C 48 --d $d --T 240000 >> $o 2>&1 || { echo "bench failed" >> $o; exit 1; }
  BC_RU_STRIP=0 timeout -k 10 120 python tools/ru_bench.py --precision h3 --iters 5 --lazy --C 48 --d $d --T 240000 >> $o 2>&1 || { echo "bench failed" >> $o; exit 1; }
done
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-x6 > gpurun_out/r03c_bench.json 2> gpurun_out/r03c_bench.err || { echo "bench.py failed $?" >> $o; exit 1; }
timeout -k 10 120 python -u tools/isa_repro/run_chain_probe.py > gpurun_out/chain_probe_gaps.txt 2>&1
echo done >> $o
