#!/bin/bash
# A/B on one box (old = a41dd07 library in gpurun_ab/old): the h3 config-2 line and the bf16 config-5 line
set -u
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
for rep in 1; do
  for v in old new; do
    if [ $v = old ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/old; else unset BIGCODEC_LIB_DIR; fi
    for cfg in "--precision h3" "--config 5" "--precision x6"; do
      timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 $cfg > $O/b.json 2>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
      python -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', '$cfg', d['value'], d['ms_per_step'], r.get('probe_bf16_tflops'), [(k['kernel'][:44], k['ms_per_step']) for k in r.get('kernels_top', [])[:4]])" >> $O/ab.txt
    done
  done
done
cat $O/ab.txt
echo done
