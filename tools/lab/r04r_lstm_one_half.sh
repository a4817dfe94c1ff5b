#!/bin/bash
# Round 4: the persistent ResLSTM runs a launch of <= 16 clips as half 0 alone (BC_LSTM_ONE_HALF) -- tests, then
# small-batch timing with and without it.
set -u
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_streaming.py -x -v --timeout 300 --timeout-method thread -k "lstm or stream" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "FAIL|Error|assert" $O/tests.txt | head -20; exit 1; }
tail -1 $O/tests.txt
for oh in 1 0; do
  for b in 1 4 16; do
    BC_LSTM_ONE_HALF=$oh timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 2 --no-cpu-baseline --no-x6 > $O/b${b}_$oh.json 2> $O/b${b}_$oh.err || { echo "b$b failed $?"; tail -5 $O/b${b}_$oh.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b${b}_$oh.json').read().strip().splitlines()[-1]);print('one_half=$oh B=$b x 10 s', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/step')"
  done
done
for oh in 1 0; do
  BC_LSTM_ONE_HALF=$oh timeout -k 10 300 python tools/stream_bench.py --decode --B 16 --chunk 1000 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
  BC_LSTM_ONE_HALF=$oh timeout -k 10 300 python tools/stream_bench.py --B 16 --chunk 4800 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
done
cat $O/stream.txt | grep stream
