#!/bin/bash
# Round 4: latency-side numbers -- config 2's encode + VQ at small batches (1, 4, 16 clips of 10 s; 1 clip of 1 s).
set -u
O=gpurun_out/r04q
mkdir -p $O
for b in 1 4 16; do
  timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 2 --no-cpu-baseline --no-x6 > $O/b$b.json 2> $O/b$b.err || { echo "b$b failed $?"; tail -5 $O/b$b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b$b.json').read().strip().splitlines()[-1]);print('B=$b x 10 s', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/step')"
done
timeout -k 10 300 python bench.py --batch 1 --seconds 1 --steps 20 --warmup 3 --no-cpu-baseline --no-x6 > $O/b1s1.json 2> $O/b1s1.err || { echo "b1s1 failed $?"; tail -5 $O/b1s1.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b1s1.json').read().strip().splitlines()[-1]);print('B=1 x 1 s', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/step')"
