#!/bin/bash
# Work-skipping ablation of the phase-decomposed strided convs on the 16-wave h3 tile (BC_X6_DEBUG bits: 1 no A copies,
# 2 no B loads, 4 no B stores, 8 no epilogue; BIGCODEC_ABLATION build under gpurun_abl/; timing only, wrong results).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
for dbg in 0 1 2 4 8 6 15; do
  echo "== dbg $dbg" >> $O/strided_ablation.txt
  BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_X6_DEBUG=$dbg timeout -k 10 120 python tools/conv_bench.py --precision h3 --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake --cfg 5322 --iters 5 >> $O/strided_ablation.txt 2>&1 || exit 1
  BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_X6_DEBUG=$dbg timeout -k 10 120 python tools/conv_bench.py --precision h3 --cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake --cfg 2322 --iters 5 >> $O/strided_ablation.txt 2>&1 || exit 1
  BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_X6_DEBUG=$dbg timeout -k 10 120 python tools/conv_bench.py --precision h3 --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake --cfg 322 --iters 5 >> $O/strided_ablation.txt 2>&1 || exit 1
done
grep -E "==|Cin" $O/strided_ablation.txt | sed 's/conv1d_x6_kernel//'
echo done
