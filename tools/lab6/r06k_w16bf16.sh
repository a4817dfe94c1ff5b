#!/bin/bash
# round 6: the bf16 (P = 1) variant of the 16-wave C = 192 unit (config 5): its tests, then config 5 with the C = 192
# units in one launch (default) against two launches (BC_RU_W16=0), same library, alternating
set -u
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -rA --timeout 300 --timeout-method thread \
  -k "fused_bf16 or w16 or bf16" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED|max" $O/tests.txt | head -30; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for v in 0 1; do
    BC_RU_W16=$v timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/c5_w$v.$rep.json 2>$O/c5_w$v.$rep.err || { echo "bench failed"; tail $O/c5_w$v.$rep.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/c5_w$v.$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('w16=$v rep $rep', d['value'], d['ms_per_step'], d.get('parity', {}))
for k in r['kernels_top'][:8]: print('   ', k['kernel'][:50], k['launches_per_step'], k['ms_per_step'])"
  done
done
echo done
