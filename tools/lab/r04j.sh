#!/bin/bash
# h3 / bf16 pointwise tile A/B after the 16-byte staging: 192 x 128 (two workgroups per CU) vs the 16-wave 192 x 256.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
for shape in "--cin 384 --cout 384 --k 1 --T 30000 --res --dual" "--cin 768 --cout 768 --k 1 --T 6000 --res --dual" "--cin 384 --cout 384 --k 1 --T 30000 --snake" "--cin 192 --cout 192 --k 1 --T 60000 --res --dual"; do
  timeout -k 10 120 python tools/conv_bench.py --iters 10 --precision h3 --cfg 314,322 $shape >> $O/pw_tiles.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/conv_bench.py --iters 10 --precision bf16 --cfg 214,222 $shape >> $O/pw_tiles.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/pw_tiles.txt | sed 's/conv1d_x6_kernel//'
