#!/bin/bash
# x6 strided (phase-decomposed) encoder convs: the 256 x 256 tile, the register-A tile and the 16-wave tile per shape
set -u
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python tools/conv_bench.py --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake --cfg 5121,5120,5122 >> $O/s.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/conv_bench.py --cin 768 --cout 1536 --k 10 --s 5 --T 1200 --snake --cfg 5120,5121,5122 >> $O/s.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/conv_bench.py --cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake --cfg 2122,2120,2121 >> $O/s.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/conv_bench.py --cin 96 --cout 192 --k 4 --s 2 --T 60000 --snake --cfg 2122,2120 >> $O/s.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/s.txt
echo done
