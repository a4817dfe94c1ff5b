#!/bin/bash
# Round 3: the decoder's transposed convs through bc_convT1d_fwd_ws (contiguous phase rows + interleave) -- convT /
# op / token / model tests, the decoder layer profile, configs 3 and 6.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03w_convt.txt; : > $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py tests/test_gpu_tokens.py -k "conv_transpose or convT or token or opcheck or ops" -x -q --timeout 200 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
timeout -k 10 200 python tools/layer_profile.py --precision h3 --decode 2>&1 | grep -v amdgpu.ids | head -12 >> $o || { echo "layers failed" >> $o; exit 1; }
for c in 3 6; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 --config $c > gpurun_out/cvt_c$c.json 2> gpurun_out/cvt_c$c.err || { echo "bench failed" >> $o; exit 1; }
  python -c "
import json
d = json.loads(open('gpurun_out/cvt_c$c.json').read().strip().splitlines()[-1])
print('config $c', d['value'], d['ms_per_step'], str(d.get('parity'))[:300])" >> $o
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_model.py -x -q --timeout 400 --timeout-method thread >> $o 2>&1 || { echo "full tests failed $?" >> $o; exit 1; }
echo done >> $o
