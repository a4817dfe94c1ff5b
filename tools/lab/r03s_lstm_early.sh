#!/bin/bash
# Round 3: the persistent ResLSTM's deferred publish flag set after k-step 0 (BC_LSTM_EARLY_FLAG = 1, default)
# instead of after all of the next half-step's MFMAs (0): LSTM / streaming / full-size tests, stamped timelines,
# configs 2 and 5 both ways.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03s_lstm_early.txt; : > $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_streaming.py -k "reslstm or stream" -x -q --timeout 200 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
for e in 0 1; do
  for B in 64 32; do
    BC_LSTM_EARLY_FLAG=$e BC_LSTM_SEQ_STAMPS=1 timeout -k 10 120 python tools/lstm_bench.py --precision h3 --B $B --T 1200 >> $o 2>&1 || { echo "failed B=$B" >> $o; exit 1; }
  done
done
for e in 0 1; do
  for c in 2 5; do
    BC_LSTM_EARLY_FLAG=$e timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 --config $c > gpurun_out/early_c${c}_$e.json 2> gpurun_out/early_c${c}_$e.err || { echo "bench failed" >> $o; exit 1; }
    python -c "
import json
d = json.loads(open('gpurun_out/early_c${c}_$e.json').read().strip().splitlines()[-1])
print('EARLY=$e config $c', d['value'], d['ms_per_step'], d.get('parity'))" >> $o
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_model.py -x -q --timeout 400 --timeout-method thread >> $o 2>&1 || { echo "full tests failed $?" >> $o; exit 1; }
echo done >> $o
