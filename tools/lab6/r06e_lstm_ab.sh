#!/bin/bash
# round 6: x6 ResLSTM with the fp32 h_t hand-off (split into bf16 planes by every consumer) against the session-start
# library (gpurun_ab/base: three bf16 planes handed off), same box, alternating; then the x6 bench line of each
set -u
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/base; else unset BIGCODEC_LIB_DIR; fi
    echo "$v $rep: $(timeout -k 10 120 python tools/lstm_bench.py --H 1536 --B 64 --T 1200 --precision x6 --iters 5 2>&1 | grep -v amdgpu.ids | tail -1)" | tee -a $O/lstm_ab.txt
  done
done
for v in base new; do
  if [ $v = base ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/base; else unset BIGCODEC_LIB_DIR; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/bench_$v.json 2>$O/bench_$v.err || { echo "bench failed"; tail $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench $v', d['value'], d['ms_per_step'], r['probe_bf16_tflops'], d['parity']['vs_reference_fixture']['index_mismatches'])
for k in r['kernels_top'][:6]: print('   ', k['kernel'][:50], k['launches_per_step'], k['ms_per_step'])"
done
echo done
