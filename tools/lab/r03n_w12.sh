#!/bin/bash
# Round 3: the 12-wave 192 x 256 tile (125: 64 x 64 per wave, three waves per SIMD) against the 16-wave tile
# (122) -- bit-identity tests, per-shape timings at the config-2 / config-5 shapes, then config 2 and 5 with
# BC_X6_W12 = 0 / 31.  One GPU process per line; the first failure ends the script.
set -u
mkdir -p gpurun_out
o=gpurun_out/r03n_w12.txt; : > $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "tiles_8_vs_16" -x -q --timeout 120 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
run() { timeout -k 10 120 python tools/conv_bench.py --iters 5 "$@" >> $o 2>&1 || { echo "failed: $*" >> $o; exit 1; }; }
for pr in h3 bf16; do
  b=3; [ $pr = bf16 ] && b=2
  run --precision $pr --cfg ${b}22,${b}25 --cin 192 --cout 192 --k 7 --d 3 --T 60000 --B 64 --snake
  run --precision $pr --cfg ${b}22,${b}25 --cin 384 --cout 384 --k 7 --d 9 --T 30000 --B 64 --snake
  run --precision $pr --cfg ${b}22,${b}25 --cin 768 --cout 768 --k 7 --d 3 --T 6000 --B 64 --snake
  run --precision $pr --cfg 5${b}22,5${b}25 --cin 384 --cout 768 --k 10 --s 5 --T 6000 --B 64 --snake
  run --precision $pr --cfg 2${b}22,2${b}25 --cin 192 --cout 384 --k 4 --s 2 --T 30000 --B 64 --snake
  run --precision $pr --cfg ${b}22,${b}25 --cin 192 --cout 192 --k 1 --T 60000 --B 64 --res --snake --dual
done
for w in 0 31; do
  BC_X6_W12=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 > gpurun_out/w12_bench_c2_$w.json 2> gpurun_out/w12_bench_c2_$w.err || { echo "bench failed" >> $o; exit 1; }
  BC_X6_W12=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 --config 5 > gpurun_out/w12_bench_c5_$w.json 2> gpurun_out/w12_bench_c5_$w.err || { echo "bench5 failed" >> $o; exit 1; }
  python -c "
import json
for c in (2, 5):
    d = json.loads(open(f'gpurun_out/w12_bench_c{c}_$w.json').read().strip().splitlines()[-1])
    print('W12=$w config', c, d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])" >> $o
done
echo done >> $o
