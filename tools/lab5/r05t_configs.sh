#!/bin/bash
# the other BASELINE configs' bench lines on the final library (no CPU baseline)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
for c in 3 4 5 6; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_config$c.json 2> $O/bench_config$c.err || { echo "config $c failed $?"; tail $O/bench_config$c.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_config$c.json').read().strip().splitlines()[-1])
print($c, d['value'], d['ms_per_step'], d.get('dtype'), d['roofline'].get('probe_bf16_tflops'), json.dumps(d.get('parity'))[:200])"
done
echo done
