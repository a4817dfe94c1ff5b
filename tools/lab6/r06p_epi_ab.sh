#!/bin/bash
# round 6: the x6 16-wave tile's epilogue in two passes of three m-tiles (RPSX 3) instead of three of two, for the
# 16-byte-staging kernels (gpurun_ab/exp) against the product library, alternating on one box
set -u
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
run() { timeout -k 10 120 python tools/conv_bench.py "$@" --iters 10 2>&1 | grep -v amdgpu.ids | tail -1 | sed 's/.*): //'; }
for rep in 1 2 3; do
  for v in base exp; do
    if [ $v = exp ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/exp; else unset BIGCODEC_LIB_DIR; fi
    echo "$v rep $rep | pw384 $(run --cin 384 --cout 384 --k 1 --T 30000 --B 64 --res --dual) | pw768 $(run --cin 768 --cout 768 --k 1 --T 6000 --B 64 --res --dual) | k7_384 $(run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --B 64 --snake)" | tee -a $O/ab.txt
  done
done
for v in base exp base exp; do
  if [ $v = exp ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/exp; else unset BIGCODEC_LIB_DIR; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/bench_$v.json 2>$O/bench_$v.err || { echo "bench failed"; tail $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench $v', d['value'], d['ms_per_step'], d['parity']['vs_reference_fixture']['index_mismatches'])
for k in r['kernels_top'][:7]: print('   %-58s %2d %8.3f' % (k['kernel'][:58], k['launches_per_step'], k['ms_per_step']))" | tee -a $O/ab.txt
done
echo done
