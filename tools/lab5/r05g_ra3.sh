#!/bin/bash
# register-A x6 conv: the remaining x6 conv tests, per-shape timing 122 vs 120, layer profile, x6 bench
set -u
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "(narrow and x6) or k7_tiles_large or (conv_transpose and x6)" --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED|passed|failed" $O/tests.txt | tail -20; exit 1; }
tail -1 $O/tests.txt
run() { timeout -k 10 120 python tools/conv_bench.py "$@" >> $O/conv.txt 2>&1 || { echo "conv bench failed $?"; tail $O/conv.txt; exit 1; }; }
run --cin 192 --cout 192 --k 7 --d 9 --T 60000 --snake --cfg 122,120
run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake --cfg 122,120
run --cin 768 --cout 768 --k 7 --d 1 --T 6000 --snake --cfg 122,120
run --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake --cfg 5121,5122,5120
run --cin 768 --cout 1536 --k 10 --s 5 --T 1200 --cfg 5122,5120
run --cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake --cfg 2122,2120
run --cin 96 --cout 192 --k 4 --s 2 --T 60000 --snake --cfg 2122,2120
grep -v amdgpu.ids $O/conv.txt
timeout -k 10 300 python tools/layer_profile.py --precision x6 > $O/layers_x6.txt 2>&1 || { echo "layers failed $?"; exit 1; }
head -30 $O/layers_x6.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h3 > $O/bench.json 2> $O/bench.err || { echo "bench failed $?"; tail $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('x6', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], d['parity']['vs_reference_fixture']['index_mismatches'])
for k in r['kernels_top']: print(k)
"
echo done
