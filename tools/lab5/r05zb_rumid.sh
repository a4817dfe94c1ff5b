#!/bin/bash
# ResidualUnit phase 1: the next step's copy and loads before m-tile 1 (current) against gpurun_ab/head, alternating
set -u
export TMPDIR=/tmp
O=gpurun_out/r05zb
mkdir -p $O
for rep in 1 2; do
  for v in head cur; do
    if [ $v = head ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/head; else unset BIGCODEC_LIB_DIR; fi
    for a in "--C 48 --d 3 --T 240000 --precision x6" "--C 96 --d 3 --T 120000 --precision x6" "--C 96 --d 3 --T 120000 --precision h3" "--C 48 --d 3 --T 720000 --B 32 --precision bf16" "--C 96 --d 9 --T 360000 --B 32 --precision bf16"; do
      echo -n "$v " >> $O/m.txt
      timeout -k 10 120 python tools/ru_bench.py $a --lazy --dual 2>&1 | grep "^resunit" >> $O/m.txt || exit 1
    done
  done
done
unset BIGCODEC_LIB_DIR
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "resunit or strip" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED" $O/tests.txt | head; exit 1; }
tail -1 $O/tests.txt
cat $O/m.txt
echo done
