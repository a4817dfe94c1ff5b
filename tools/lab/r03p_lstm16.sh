#!/bin/bash
# Round 3: the persistent ResLSTM with halves of 16 clips for launches of <= 32 clips (config 5: 32 per GPU):
# LSTM kernel tests, then config 5 with BC_LSTM_NH16 = 0 (halves of 32, half 1 empty) and 1, and config 2.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03p_lstm16.txt; : > $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "reslstm" -x -q --timeout 200 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
for v in 0 1; do
  BC_LSTM_NH16=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 --config 5 > gpurun_out/lstm16_c5_$v.json 2> gpurun_out/lstm16_c5_$v.err || { echo "bench5 failed" >> $o; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/lstm16_c5_$v.json').read().strip().splitlines()[-1])
print('NH16=$v config 5', d['value'], d['ms_per_step'], d.get('parity'))" >> $o
done
timeout -k 10 200 python tools/layer_profile.py --precision bf16 --batch 32 --seconds 30 2>&1 | grep -v amdgpu.ids | head -4 >> $o || { echo "layers failed" >> $o; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_full_size.py -x -q --timeout 300 --timeout-method thread -k "bf16 or 30s" >> $o 2>&1 || { echo "model tests failed $?" >> $o; exit 1; }
echo done >> $o
