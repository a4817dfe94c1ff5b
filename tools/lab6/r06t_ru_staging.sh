#!/bin/bash
# round 6: the one-launch unit's staging skips the zero padding (pairs past Cin: zeros stored, no Snake / split; 32-column
# passes past ncol: no Snake) -- unit tests, then the units against the previous library (gpurun_ab/prev), alternating
set -u
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -rA --timeout 300 --timeout-method thread \
  -k "resunit" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ru() { timeout -k 10 100 python tools/ru_bench.py "$@" --lazy --iters 10 2>&1 | grep resunit | sed 's/.*: //'; }
for rep in 1 2 3; do
  for v in prev new; do
    if [ $v = prev ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/prev; else unset BIGCODEC_LIB_DIR; fi
    echo "$v $rep | x6 48 d1 $(ru --C 48 --d 1 --T 240000 --precision x6) | x6 48 d9 $(ru --C 48 --d 9 --T 240000 --precision x6) | x6 96 d3 $(ru --C 96 --d 3 --T 120000 --precision x6) | bf16 48 d3 $(ru --C 48 --d 3 --T 240000 --precision bf16)" | tee -a $O/ab.txt
  done
done
for v in prev new prev new; do
  if [ $v = prev ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/prev; else unset BIGCODEC_LIB_DIR; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/bench_$v.json 2>$O/bench_$v.err || { echo "bench failed"; tail $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench $v', d['value'], d['ms_per_step'], d['parity']['vs_reference_fixture']['index_mismatches'])
for k in r['kernels_top'][:8]: print('   %-58s %2d %8.3f' % (k['kernel'][:58], k['launches_per_step'], k['ms_per_step']))" | tee -a $O/ab.txt
done
echo done
