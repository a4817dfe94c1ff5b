#!/bin/bash
# round 6: first-round stagger of the x6 conv tile (BC_X6_STAGGER = s_sleep(127) count for half of each XCD's first
# 256 workgroups): pointwise C = 384 / 768 (residual + dual output) and k7 C = 384 / 192 (Snake epilogue), alternating
set -u
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
run() { timeout -k 10 120 python tools/conv_bench.py "$@" --iters 10 2>&1 | grep -v amdgpu.ids | tail -1 | sed 's/.*): //'; }
for rep in 1 2; do
  for st in 0 4 8 16 32; do
    export BC_X6_STAGGER=$st
    echo "st $st rep $rep | pw384 $(run --cin 384 --cout 384 --k 1 --T 30000 --B 64 --res --dual) | pw768 $(run --cin 768 --cout 768 --k 1 --T 6000 --B 64 --res --dual) | k7_384 $(run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --B 64 --snake) | k7_768 $(run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --B 64 --snake)" | tee -a $O/stagger.txt
  done
done
echo done
