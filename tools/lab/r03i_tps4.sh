#!/bin/bash
# bf16 16-wave k7 tile: 4 taps per K-step (default) vs 2 (BC_X6_TPS4=0), config-5 shapes; then its parity tests
set -u
mkdir -p gpurun_out/r03i
o=gpurun_out/r03i/tps4.txt
for shp in "--cin 192 --cout 192 --k 7 --d 3 --T 180000" "--cin 384 --cout 384 --k 7 --d 3 --T 90000" "--cin 768 --cout 768 --k 7 --d 9 --T 18000"; do
  for t in 1 0; do
    BC_X6_TPS4=$t timeout -k 10 120 python tools/conv_bench.py --precision bf16 --B 8 --iters 5 --snake $shp >> $o 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "8_vs_16 or bf16" > gpurun_out/r03i/tests.log 2>&1 || { tail -30 gpurun_out/r03i/tests.log; exit 1; }
tail -2 gpurun_out/r03i/tests.log
timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03i/bench5.json 2> gpurun_out/r03i/bench5.err || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/r03i/bench5.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['mismatch_rate'], d['roofline']['kernel'], d['roofline']['frac'])
for k in d['roofline']['kernels_top'][:6]: print(k)
"
