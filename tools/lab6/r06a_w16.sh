#!/bin/bash
# round 6: first GPU run of the one-launch C = 192 x6 ResidualUnit (resunit_w16.hip): its tests, unit timing, and the
# config-2 line with and without it (BC_RU_W16=0: the two-launch units), same box
set -u
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "w16_c192 or (resunit_fused and x6)" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
grep -E "passed|failed|w16 C=192" $O/tests.txt | tail -12
for d in 1 3 9; do
  timeout -k 10 100 python tools/ru_bench.py --C 192 --d $d --T 60000 --precision x6 --dual >> $O/ru.txt 2>&1 || { echo "ru failed"; tail $O/ru.txt; exit 1; }
  timeout -k 10 100 python tools/ru_bench.py --C 192 --d $d --T 60000 --precision x6 --dual --lazy >> $O/ru.txt 2>&1 || { echo "ru failed"; tail $O/ru.txt; exit 1; }
done
grep -v amdgpu.ids $O/ru.txt
for v in on off on; do
  if [ $v = off ]; then export BC_RU_W16=0; else unset BC_RU_W16; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/bench_$v.json 2>$O/bench_$v.err || { echo "bench failed"; tail $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench $v', d['value'], d['ms_per_step'], r['probe_bf16_tflops'], d['parity']['vs_reference_fixture']['index_mismatches'])
for k in r['kernels_top']: print('   ', k['kernel'][:60], k['launches_per_step'], k['ms_per_step'], k['frac_mfma_spec'])"
done
echo done
