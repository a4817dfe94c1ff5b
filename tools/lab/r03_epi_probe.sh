#!/bin/bash
# Round 3: what the Snake in the k7 epilogue costs (k7 C = 192 / 384 / 768 with and without the output Snake) and
# the pointwise convs with / without it (h3, B = 64, the config-2 shapes).  One GPU process per line.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03_epi_probe.txt; : > $o
run() { timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 10 "$@" >> $o 2>&1 || { echo "failed: $*" >> $o; exit 1; }; }
run --cin 192 --cout 192 --k 7 --d 3 --T 60000
run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake
run --cin 384 --cout 384 --k 7 --d 3 --T 30000
run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake
run --cin 768 --cout 768 --k 7 --d 3 --T 6000
run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake
run --cin 192 --cout 192 --k 1 --T 60000 --res
run --cin 192 --cout 192 --k 1 --T 60000 --res --dual
run --cin 384 --cout 384 --k 1 --T 30000 --res
run --cin 384 --cout 384 --k 1 --T 30000 --res --dual
run --cin 768 --cout 768 --k 1 --T 6000 --res --dual
echo done >> $o
