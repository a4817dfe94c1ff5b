#!/bin/bash
# Round 4: narrow-launch tiles (bc_conv1d_select_cfg_n) -- tests, stream / small-batch timing with and without.
set -u
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_streaming.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "narrow or stream or model" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "FAIL|Error|assert" $O/tests.txt | head -20; exit 1; }
tail -1 $O/tests.txt
for nw in 1 0; do
  BC_X6_NARROW=$nw timeout -k 10 300 python tools/stream_bench.py --decode --B 16 --chunk 1000 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
  BC_X6_NARROW=$nw timeout -k 10 300 python tools/stream_bench.py --chunk 4800 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
  BC_X6_NARROW=$nw timeout -k 10 300 python tools/stream_bench.py --chunk 1200 --B 16 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
  echo "narrow=$nw" >> $O/stream.txt
done
grep -E "stream|narrow" $O/stream.txt
