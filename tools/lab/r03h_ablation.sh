#!/bin/bash
# Main-loop ablation of the 16-wave k7 tile in bf16 and h3 (BC_X6_DEBUG bits: 1 no A copies, 2 no B loads, 4 no B
# stores, 8 no epilogue), on an ablation build placed under gpurun_abl/ (BIGCODEC_ABLATION=1).  Timing only.
set -u
mkdir -p gpurun_out/r03h
o=gpurun_out/r03h/ablation.txt
for dbg in 0 1 2 4 8 6 15; do
  echo "== dbg $dbg" >> $o
  for pc in "bf16 222" "h3 322"; do
    set -- $pc
    BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_X6_DEBUG=$dbg timeout -k 10 120 python tools/conv_bench.py --precision $1 --cin 384 --cout 384 --k 7 --d 3 --T 90000 --B 8 --snake --cfg $2 --iters 5 >> $o 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $o
