#!/bin/bash
# Round 3: the Cout = 1 conv on the 16 x 256 tile -- conv / model / full-size tests and configs 3, 6.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03y_cout1_check.txt; : > $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_tokens.py tests/test_gpu_full_size.py -k "conv1d or model or token or config3 or layers" -x -q --timeout 300 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
for c in 3 6; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 --config $c > gpurun_out/c1_c$c.json 2> gpurun_out/c1_c$c.err || { echo "bench failed" >> $o; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/c1_c$c.json').read().strip().splitlines()[-1])
print('config $c', d['value'], d['ms_per_step'], str(d.get('parity'))[:200], d['roofline'].get('probe_bf16_tflops'))" >> $o
done
echo done >> $o
