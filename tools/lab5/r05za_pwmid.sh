#!/bin/bash
# pointwise path: the next chunk's copy and loads after the first m-tile (current) against gpurun_ab/head, alternating
set -u
export TMPDIR=/tmp
O=gpurun_out/r05za
mkdir -p $O
for rep in 1 2; do
  for v in head cur; do
    if [ $v = head ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/head; else unset BIGCODEC_LIB_DIR; fi
    for p in x6 h3 bf16; do
      for shp in "--cin 192 --cout 192 --T 60000" "--cin 384 --cout 384 --T 30000" "--cin 768 --cout 768 --T 6000"; do
        echo -n "$v $p " >> $O/m.txt
        timeout -k 10 120 python tools/conv_bench.py $shp --k 1 --res --snake --dual --precision $p 2>&1 | grep "^Cin" >> $O/m.txt || exit 1
      done
    done
  done
done
unset BIGCODEC_LIB_DIR
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "b4_staging or narrow or presplit or conv1d" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED" $O/tests.txt | head; exit 1; }
tail -1 $O/tests.txt
cat $O/m.txt
echo done
