#!/bin/bash
# Round 4: tile sweep on narrow shapes (streaming chunks / small batches): which tile wins when B * T is small.
set -u
O=gpurun_out/r04s
mkdir -p $O
run() { timeout -k 10 240 python tools/conv_bench.py --precision h3 --cfg all --iters 20 "$@" >> $O/sweep.txt 2>&1 || { echo "failed $? on $*"; tail -3 $O/sweep.txt; exit 1; }; }
run --cin 768 --cout 768 --k 7 --d 1 --T 25 --B 16 --snake
run --cin 384 --cout 384 --k 7 --d 3 --T 125 --B 16 --snake
run --cin 1024 --cout 1536 --k 7 --d 1 --T 5 --B 16
run --cin 768 --cout 768 --k 7 --d 9 --T 120 --B 64 --snake
run --cin 1536 --cout 1536 --k 7 --d 1 --T 24 --B 64
grep "best cfg" $O/sweep.txt
