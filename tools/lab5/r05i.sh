#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "resunit and x6" --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED|passed|failed" $O/tests.txt | tail -20; exit 1; }
tail -1 $O/tests.txt
for d in 1 3 9; do
  for tps in 1 2; do
    BC_RU_TPS=$tps timeout -k 10 100 python tools/ru_bench.py --C 48 --d $d --T 240000 --precision x6 --lazy >> $O/ru.txt 2>&1 || { echo "ru bench failed $?"; tail $O/ru.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/ru.txt
for p in x6 h3; do
  BC_LSTM_SEQ_STAMPS=1 timeout -k 10 200 python tools/lstm_bench.py --precision $p --layers 1 > $O/stamps_$p.txt 2>&1 || { echo "lstm $p failed $?"; exit 1; }
  grep -v amdgpu.ids $O/stamps_$p.txt
done
echo done
