#!/bin/bash
# bf16 (config 5) tile sweep over the encoder's conv shapes at 30 s clips (per-clip T as in config 5, B = 8):
# every tile via tools/conv_bench.py --cfg all; results -> gpurun_out/r03g/sweep.txt
set -u
mkdir -p gpurun_out/r03g
o=gpurun_out/r03g/sweep.txt
run() { timeout -k 10 240 python tools/conv_bench.py --precision bf16 --B 8 --iters 3 --cfg all "$@" >> $o 2>&1 || { echo "failed: $*"; exit 1; }; }
run --cin 192 --cout 192 --k 7 --d 3 --T 180000 --snake
run --cin 384 --cout 384 --k 7 --d 3 --T 90000 --snake
run --cin 768 --cout 768 --k 7 --d 9 --T 18000 --snake
run --cin 96 --cout 192 --k 4 --s 2 --T 180000 --snake
run --cin 192 --cout 384 --k 4 --s 2 --T 90000 --snake
run --cin 384 --cout 768 --k 10 --s 5 --T 18000 --snake
run --cin 768 --cout 1536 --k 10 --s 5 --T 3600 --snake
run --cin 192 --cout 192 --k 1 --T 180000 --res --dual
run --cin 384 --cout 384 --k 1 --T 90000 --res --dual
run --cin 768 --cout 768 --k 1 --T 18000 --res --dual
grep "best" $o
