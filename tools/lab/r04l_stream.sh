#!/bin/bash
# Round 4: the streaming state on bc_stream_window + one-launch ResidualUnits over context windows: GPU tests and
# an A/B against the previous stream (tools/lab/streaming_prev.py) on the causal `default` model, B = 64 x 10 s.
set -u
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_streaming.py -x -v --timeout 300 --timeout-method thread -s > $O/tests.txt 2>&1 || { echo "tests failed $?"; tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for ch in 24000 4800; do
  for v in "" "--prev"; do
    timeout -k 10 300 python tools/stream_bench.py --chunk $ch $v >> $O/bench.txt 2>&1 || { echo "bench failed $?"; tail -5 $O/bench.txt; exit 1; }
  done
done
for ch in 4000 1000; do
  for v in "" "--prev"; do
    timeout -k 10 300 python tools/stream_bench.py --decode --B 16 --chunk $ch $v >> $O/bench.txt 2>&1 || { echo "bench failed $?"; tail -5 $O/bench.txt; exit 1; }
  done
done
grep stream $O/bench.txt
