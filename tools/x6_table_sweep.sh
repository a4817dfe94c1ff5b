#!/bin/bash
# x6 (three bf16 planes) tile table: the library's current choice ("c") against the wide 8-wave tiles
# (120: 192 x 256, 121: 256 x 256) and the 16-wave 192 x 256 tile (122) that the h3 / bf16 tables use, on
# every conv shape of the config-2 encoder (B = 64 x 10 s).  -> gpurun_out/x6_sweep.log
set -u
mkdir -p gpurun_out
run() { timeout -k 10 240 python tools/conv_bench.py --iters 5 --precision x6 "$@" >> gpurun_out/x6_sweep.log 2>&1 || { echo "failed $? on $*"; exit 1; }; }
run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake --cfg c,120,122
run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake --cfg c,120,122
run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake --cfg c,120,121,122
run --cin 192 --cout 192 --k 1 --T 60000 --res --dual --cfg c,114,122
run --cin 384 --cout 384 --k 1 --T 30000 --res --dual --cfg c,114,122
run --cin 768 --cout 768 --k 1 --T 6000 --res --dual --cfg c,114,122
run --cin 1536 --cout 6144 --k 1 --T 76800 --B 1 --cfg c,121,122
run --cin 48 --cout 96 --k 4 --s 2 --T 120000 --snake --cfg c,2122
run --cin 96 --cout 192 --k 4 --s 2 --T 60000 --snake --cfg c,2120,2122
run --cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake --cfg c,2120,2122
run --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake --cfg c,5120,5121,5122
run --cin 768 --cout 1536 --k 10 --s 5 --T 1200 --cfg c,5120,5121,5122
run --cin 1536 --cout 1024 --k 3 --T 1200 --cfg c,121,122
echo done
