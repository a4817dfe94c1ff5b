#!/bin/bash
# x6 C = 48 / 96 unit tiles: the two-per-CU tiles against the wider one-per-CU ones (BC_RU_CFG), taps per K-step
set -u
export TMPDIR=/tmp
O=gpurun_out/r05u
mkdir -p $O
for d in 3 9; do
  for cfg in 111 106 124; do
    for tps in 1 2; do
      BC_RU_CFG=$cfg BC_RU_TPS=$tps timeout -k 10 100 python tools/ru_bench.py --C 48 --d $d --T 240000 --precision x6 --lazy --dual --cfg $cfg >> $O/ru.txt 2>&1 || echo "cfg $cfg tps $tps failed" >> $O/ru.txt
    done
  done
  for cfg in 109 104 123; do
    BC_RU_CFG=$cfg timeout -k 10 100 python tools/ru_bench.py --C 96 --d $d --T 120000 --precision x6 --lazy --dual --cfg $cfg >> $O/ru.txt 2>&1 || echo "cfg $cfg failed" >> $O/ru.txt
  done
done
grep -v amdgpu.ids $O/ru.txt | grep -v "^Traceback\|^  File\|^    " | tail -40
echo done
