#!/bin/bash
# round 6, VERDICT r05 item 1(b): what dropping the C = 384 / 768 pointwise convs' activated second output (the next
# unit's k7 applying the Snake on load instead) would save and cost, on the BIGCODEC_ABLATION=1 build under gpurun_abl/:
#   BC_ABL_PW_RAW_ONLY=1  the dual-output pointwise launches write the raw output only (the saving)
#   BC_X6_DEBUG=32        the C = 192 unit's phase 1 stages its input without the Snake (the Snake-on-load cost)
set -u
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
L=$PWD/gpurun_abl/audiotokenization_amd
for rep in 1 2; do
  for v in base raw_only nosin; do
    E=""
    [ $v = raw_only ] && E="BC_ABL_PW_RAW_ONLY=1"
    [ $v = nosin ] && E="BC_X6_DEBUG=32"
    env $E BIGCODEC_LIB_DIR=$L timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-h3 > $O/b_$v.$rep.json 2>$O/b_$v.$rep.err || { echo "bench $v failed"; tail $O/b_$v.$rep.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/b_$v.$rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v rep $rep', d['value'], d['ms_per_step'])
for k in r['kernels_top'][:9]: print('   %-58s %2d %8.3f' % (k['kernel'][:58], k['launches_per_step'], k['ms_per_step']))" | tee -a $O/summary.txt
  done
done
for x in 0 32 0 32; do
  BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_X6_DEBUG=$x timeout -k 10 100 python tools/ru_bench.py --C 192 --d 3 --T 60000 --precision x6 --lazy --iters 10 > $O/t.txt 2>&1 || { echo "ru failed"; tail $O/t.txt; exit 1; }
  echo "w16 C=192 d=3 lazy, BC_X6_DEBUG=$x: $(grep resunit $O/t.txt)" | tee -a $O/summary.txt
done
echo done
