#!/bin/bash
# Round 3: one-launch ResidualUnit tile shapes at the encoder shapes (snake on load), default vs the new
# 123 (96 x 128 as 2 x 4 waves of 48 x 32) and 124 / 106 (bf16 C = 48: 48 x 512 / 48 x 256 tiles), then the
# bit-identity tests.  One GPU process per line; the first failure ends the script.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03m_ru_tiles.txt; : > $o
run() { timeout -k 10 120 python tools/ru_bench.py --iters 5 --lazy "$@" >> $o 2>&1 || { echo "failed: $*" >> $o; exit 1; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "tiles_bit_identical" -x -q --timeout 120 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
for d in 1 3 9; do
  run --precision h3 --C 96 --d $d --T 120000
  run --precision h3 --C 96 --d $d --T 120000 --cfg 323
  run --precision bf16 --C 96 --d $d --T 360000 --B 32
  run --precision bf16 --C 96 --d $d --T 360000 --B 32 --cfg 223
  run --precision bf16 --C 48 --d $d --T 720000 --B 32
  run --precision bf16 --C 48 --d $d --T 720000 --B 32 --cfg 224
  run --precision bf16 --C 48 --d $d --T 720000 --B 32 --cfg 206
done
run --precision x6 --C 96 --d 3 --T 120000
run --precision x6 --C 96 --d 3 --T 120000 --cfg 123
echo done >> $o
