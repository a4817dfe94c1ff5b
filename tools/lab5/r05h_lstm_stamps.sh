#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
for p in x6 h3; do
  BC_LSTM_SEQ_STAMPS=1 timeout -k 10 200 python tools/lstm_bench.py --precision $p --layers 1 > $O/stamps_$p.txt 2>&1 || { echo "lstm $p failed $?"; exit 1; }
  grep -v amdgpu.ids $O/stamps_$p.txt
done
BC_LSTM_SEQ_STAMPS=1 timeout -k 10 200 python tools/lstm_bench.py --precision x6 --layers 1 --B 1 > $O/stamps_x6_b1.txt 2>&1 || { echo "lstm b1 failed $?"; exit 1; }
grep -v amdgpu.ids $O/stamps_x6_b1.txt
echo done
