#!/bin/bash
# round 6: ablation of the one-launch C = 192 unit (resunit_w16.hip, BC_W16_DEBUG bits; needs the BIGCODEC_ABLATION=1
# build under gpurun_abl/), C = 192 d = 3, 64 x 60 000, snake on load + dual output as in the encoder flow
set -u
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
for dbg in 0 1 2 3 4 8 15 0; do
  BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_W16_DEBUG=$dbg timeout -k 10 100 python tools/ru_bench.py --C 192 --d 3 --T 60000 --precision x6 --dual --lazy --iters 10 > $O/t.txt 2>&1 || { echo "ru failed"; tail $O/t.txt; exit 1; }
  echo "dbg $dbg: $(grep resunit $O/t.txt)" | tee -a $O/abl.txt
done
for x in 1 2 4; do
  BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_X6_DEBUG=$x timeout -k 10 100 python tools/ru_bench.py --C 192 --d 3 --T 60000 --precision x6 --dual --lazy --iters 10 > $O/t.txt 2>&1 || { echo "ru failed"; tail $O/t.txt; exit 1; }
  echo "phase-1 dbg $x: $(grep resunit $O/t.txt)" | tee -a $O/abl.txt
done
echo done
