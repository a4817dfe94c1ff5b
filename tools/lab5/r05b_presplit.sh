#!/bin/bash
# x6 pre-split LSTM input projection: bit-identity tests, then layer timing on / off, then the layer profile
set -u
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "presplit or reslstm" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for ps in 1 0; do
  BC_LSTM_PRESPLIT=$ps timeout -k 10 200 python tools/lstm_bench.py --precision x6 --layers 2 > $O/lstm_ps$ps.txt 2>&1 || { echo "lstm bench failed $?"; exit 1; }
  echo "presplit=$ps"; tail -3 $O/lstm_ps$ps.txt
done
timeout -k 10 300 python tools/layer_profile.py --precision x6 > $O/layers_x6.txt 2>&1 || { echo "layers failed $?"; exit 1; }
head -3 $O/layers_x6.txt
echo done
