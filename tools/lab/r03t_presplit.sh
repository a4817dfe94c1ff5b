#!/bin/bash
# Round 3: the ResLSTM input projection on the pre-split GEMM (pw_presplit.hip) -- bit-identity and LSTM tests,
# layer timings and configs 2 / 5 with BC_LSTM_PRESPLIT = 0 / 1, then the full-size and model tests.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03t_presplit.txt; : > $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "presplit or reslstm" -x -q --timeout 200 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
for e in 0 1; do
  BC_LSTM_PRESPLIT=$e timeout -k 10 120 python tools/lstm_bench.py --precision h3 --B 64 --T 1200 --layers 2 >> $o 2>&1 || { echo "lstm bench failed" >> $o; exit 1; }
  for c in 2 5; do
    BC_LSTM_PRESPLIT=$e timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 --config $c > gpurun_out/ps_c${c}_$e.json 2> gpurun_out/ps_c${c}_$e.err || { echo "bench failed" >> $o; exit 1; }
    python -c "
import json
d = json.loads(open('gpurun_out/ps_c${c}_$e.json').read().strip().splitlines()[-1])
print('PRESPLIT=$e config $c', d['value'], d['ms_per_step'], d.get('parity'))" >> $o
  done
done
timeout -k 10 200 python tools/layer_profile.py --precision h3 2>&1 | grep -v amdgpu.ids | head -4 >> $o || { echo "layers failed" >> $o; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_model.py tests/test_gpu_streaming.py -x -q --timeout 400 --timeout-method thread >> $o 2>&1 || { echo "full tests failed $?" >> $o; exit 1; }
echo done >> $o
