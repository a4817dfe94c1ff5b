#!/bin/bash
# One-launch ResidualUnit at the encoder's C = 48 / 96 shapes, snake on load and dual output as the flow runs
# them: resunit_x6 (BC_RU_RR=0) against the default selection (resunit_rr at C = 48).  profiles/r02_ru_rr_sweep.txt
set -u
mkdir -p gpurun_out
out=gpurun_out/ru_rr_sweep.log
: > $out
for d in 1 9; do
  for rr in 0 1; do
    BC_RU_RR=$rr timeout -k 10 120 python tools/ru_bench.py --C 48 --d $d --T 240000 --lazy --dual >> $out 2>&1 || exit 1
    BC_RU_RR=$rr timeout -k 10 120 python tools/ru_bench.py --C 96 --d $d --T 120000 --lazy --dual >> $out 2>&1 || exit 1
  done
done
echo done
