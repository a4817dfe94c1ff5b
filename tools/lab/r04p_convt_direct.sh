#!/bin/bash
# Round 4: ConvTranspose1d -- per-phase workspace + interleave pass vs direct strided stores, by stride (config 6).
set -u
O=gpurun_out/r04p
mkdir -p $O
for m in 0 2 5; do
  BC_CONVT_DIRECT_MAXS=$m timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --no-x6 --steps 4 --warmup 1 > $O/c6_$m.json 2> $O/c6_$m.err || { echo "c6 $m failed $?"; tail -5 $O/c6_$m.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c6_$m.json').read().strip().splitlines()[-1]);print('direct<=$m', d['value'], d['ms_per_step'])"
done
for m in 0 2; do
  BC_CONVT_DIRECT_MAXS=$m timeout -k 10 300 python bench.py --config 6 --no-cpu-baseline --no-x6 --steps 4 --warmup 1 > $O/c6b_$m.json 2> $O/c6b_$m.err || { echo "c6b $m failed $?"; exit 1; }
  python -c "import json;d=json.loads(open('$O/c6b_$m.json').read().strip().splitlines()[-1]);print('again direct<=$m', d['value'], d['ms_per_step'])"
done
