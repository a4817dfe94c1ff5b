#!/bin/bash
# Persistent multi-tap conv kernel: parity (kernel + ops + model tests), then same-box A/B of BC_X6_PERSIST=1 / 0
# on the config-2 / config-5 conv shapes and the config-2 bench.
set -u
mkdir -p gpurun_out/r03l
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03l/tests.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/r03l/tests.log | head -20; tail -40 gpurun_out/r03l/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r03l/tests.log | tail -2
o=gpurun_out/r03l/ab.txt
for rep in 1 2; do
  for pr in h3 bf16; do
    for shp in "--cin 384 --cout 384 --k 7 --d 3 --T 30000 --B 64 --snake" "--cin 192 --cout 192 --k 7 --d 3 --T 60000 --B 64 --snake" \
               "--cin 768 --cout 768 --k 7 --d 9 --T 6000 --B 64 --snake" "--cin 384 --cout 768 --k 10 --s 5 --T 6000 --B 64 --snake"; do
      for p in 1 0; do
        echo "persist $p" >> $o
        BC_X6_PERSIST=$p timeout -k 10 120 python tools/conv_bench.py --precision $pr --iters 5 $shp >> $o 2>&1 || exit 1
      done
    done
  done
done
python - <<'PY'
import re, collections
d = collections.defaultdict(list)
tag = None
for l in open("gpurun_out/r03l/ab.txt"):
    if l.startswith("persist"):
        tag = l.split()[1]; continue
    m = re.search(r"Cin=(\d+) Cout=(\d+) k=(\d+) s=(\d+).*\((conv1d_x6_kernel<[^>]*>)\): ([\d.]+) ms  ([\d.]+) TFLOP", l)
    if m:
        d[(m.group(5), m.group(1), m.group(3), m.group(4), tag)].append((float(m.group(6)), float(m.group(7))))
for k in sorted({k[:4] for k in d}):
    n, o = min(d[k + ("1",)]), min(d[k + ("0",)])
    print(f"{k[0]} Cin={k[1]} k={k[2]} s={k[3]}: persistent {n[0]:.3f} ms ({n[1]:.0f} TF) vs one tile per workgroup {o[0]:.3f} ms ({o[1]:.0f} TF): {n[0]/o[0]:.3f}")
PY
for p in 1 0; do
  BC_X6_PERSIST=$p timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-x6 > gpurun_out/r03l/bench2_p$p.json 2> gpurun_out/r03l/bench2_p$p.err || exit 1
done
BC_X6_PERSIST=1 timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03l/bench5_p1.json 2> gpurun_out/r03l/bench5_p1.err || exit 1
python -c "
import json
for f in ['bench2_p1','bench2_p0','bench5_p1']:
    d=json.loads(open('gpurun_out/r03l/'+f+'.json').read().strip().splitlines()[-1]); r=d['roofline']
    print(f, d['value'], d['ms_per_step'], r['kernel'], r['frac'], r['avg_launch_ms'])
"
