#!/bin/bash
# Same-box A/B of the conv epilogue: coefficients staged in LDS (this tree) vs read from memory inside the
# epilogue (the previous build, placed under gpurun_abl/), interleaved, 3 repeats per shape.
set -u
mkdir -p gpurun_out/r03k
o=gpurun_out/r03k/ab.txt
for rep in 1 2 3; do
  for pr in h3 bf16; do
    for shp in "--cin 384 --cout 384 --k 7 --d 3 --T 90000 --snake" "--cin 192 --cout 192 --k 1 --T 180000 --res --dual" \
               "--cin 384 --cout 384 --k 1 --T 90000 --res --dual" "--cin 768 --cout 768 --k 1 --T 18000 --res --dual"; do
      echo "new $rep" >> $o
      timeout -k 10 120 python tools/conv_bench.py --precision $pr --B 8 --iters 5 $shp >> $o 2>&1 || exit 1
      echo "old $rep" >> $o
      BIGCODEC_PKG_ROOT=$PWD/gpurun_abl timeout -k 10 120 python tools/conv_bench.py --precision $pr --B 8 --iters 5 $shp >> $o 2>&1 || exit 1
    done
  done
done
python - <<'PY'
import re, collections
d = collections.defaultdict(list)
tag = None
for l in open("gpurun_out/r03k/ab.txt"):
    if l.startswith(("new", "old")):
        tag = l.split()[0]; continue
    m = re.search(r"Cin=(\d+) Cout=(\d+) k=(\d+).*\((conv1d_x6_kernel<[^>]*>)\): ([\d.]+) ms", l)
    if m:
        d[(m.group(4), m.group(1), m.group(3), tag)].append(float(m.group(5)))
keys = sorted({k[:3] for k in d})
for k in keys:
    n, o = d[k + ("new",)], d[k + ("old",)]
    print(f"{k[0]} C={k[1]} k={k[2]}: new {min(n):.3f} old {min(o):.3f} ms (min of {len(n)}), ratio {min(n)/min(o):.3f}")
PY
