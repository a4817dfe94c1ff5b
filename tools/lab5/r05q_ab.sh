#!/bin/bash
# A/B on one box: the round-5 library before this session's changes (gpurun_ab/old, built from a41dd07) against the
# current one, alternating, on the unit / conv shapes and the x6 bench line
set -u
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/old; else unset BIGCODEC_LIB_DIR; fi
    echo "== $v rep $rep" >> $O/ab.txt
    for a in "--C 48 --d 3 --T 240000" "--C 96 --d 3 --T 120000"; do
      timeout -k 10 100 python tools/ru_bench.py $a --precision x6 --lazy --dual >> $O/ab.txt 2>&1 || { echo "ru failed"; tail $O/ab.txt; exit 1; }
    done
    for shp in "--cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake" "--cin 384 --cout 384 --T 30000 --k 1 --res --snake --dual"; do
      timeout -k 10 120 python tools/conv_bench.py $shp >> $O/ab.txt 2>&1 || { echo "conv failed"; tail $O/ab.txt; exit 1; }
    done
    timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/bench_$v$rep.json 2>$O/bench_$v$rep.err || { echo "bench failed"; tail $O/bench_$v$rep.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench_$v$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench', d['value'], d['ms_per_step'], r['probe_bf16_tflops'], [(k['kernel'][:40], k['ms_per_step']) for k in r['kernels_top']])" >> $O/ab.txt
  done
done
grep -v amdgpu.ids $O/ab.txt
echo done
