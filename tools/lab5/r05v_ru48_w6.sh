#!/bin/bash
# x6 C = 48 unit compiled for 6 waves per SIMD (80 VGPRs: three 8-wave workgroups per CU at one tap per K-step)
# against the 4-wave build, alternating on one box
set -u
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
for rep in 1 2; do
  for v in cur w6; do
    if [ $v = w6 ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/w6; else unset BIGCODEC_LIB_DIR; fi
    for d in 3 9; do
      for tps in 1 2; do
        echo -n "$v tps$tps " >> $O/ru.txt
        BC_RU_TPS=$tps timeout -k 10 100 python tools/ru_bench.py --C 48 --d $d --T 240000 --precision x6 --lazy --dual 2>&1 | grep resunit >> $O/ru.txt || { echo "failed"; exit 1; }
      done
    done
  done
done
cat $O/ru.txt
echo done
