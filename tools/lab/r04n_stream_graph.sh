#!/bin/bash
# Round 4: streaming pushes as one HIP-graph replay (StreamGraph): tests, then eager vs graph timing.
set -u
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_streaming.py -x -v --timeout 300 --timeout-method thread -s -k "graph or window" > $O/tests.txt 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for ch in 24000 4800 1200; do
  for v in "" "--graph"; do
    timeout -k 10 300 python tools/stream_bench.py --chunk $ch $v >> $O/bench.txt 2>&1 || { echo "bench failed $?"; tail -5 $O/bench.txt; exit 1; }
  done
done
for ch in 4000 1000; do
  for v in "" "--graph"; do
    timeout -k 10 300 python tools/stream_bench.py --decode --B 16 --chunk $ch $v >> $O/bench.txt 2>&1 || { echo "bench failed $?"; tail -5 $O/bench.txt; exit 1; }
  done
done
grep stream $O/bench.txt
