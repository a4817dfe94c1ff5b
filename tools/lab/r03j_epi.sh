#!/bin/bash
# Epilogue with the per-channel coefficients read up front: conv timings (compare with r03g/r03h/r03i), kernel
# parity tests, config-2 bench
set -u
mkdir -p gpurun_out/r03j
o=gpurun_out/r03j/conv.txt
for pr in h3 bf16; do
  for shp in "--cin 384 --cout 384 --k 7 --d 3 --T 90000 --snake" "--cin 192 --cout 192 --k 7 --d 3 --T 180000 --snake" \
             "--cin 192 --cout 192 --k 1 --T 180000 --res --dual" "--cin 384 --cout 384 --k 1 --T 90000 --res --dual" \
             "--cin 768 --cout 768 --k 1 --T 18000 --res --dual"; do
    timeout -k 10 120 python tools/conv_bench.py --precision $pr --B 8 --iters 5 $shp >> $o 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03j/tests.log 2>&1 || { tail -30 gpurun_out/r03j/tests.log; exit 1; }
tail -2 gpurun_out/r03j/tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-x6 > gpurun_out/r03j/bench2.json 2> gpurun_out/r03j/bench2.err || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/r03j/bench2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])
for k in d['roofline']['kernels_top'][:8]: print(k)
"
