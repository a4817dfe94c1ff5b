#!/bin/bash
# 16-wave tile workgroup order: row groups of a column tile consecutive (default) vs column tiles fastest
# (BC_X6_RASTER=1), alternating on one box
set -u
export TMPDIR=/tmp
O=gpurun_out/r05zg
mkdir -p $O
for rep in 1 2; do
  for ra in 0 1; do
    for shp in "--cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake" "--cin 384 --cout 384 --k 7 --d 9 --T 30000 --snake" "--cin 768 --cout 768 --k 7 --d 1 --T 6000 --snake" "--cin 384 --cout 384 --k 1 --T 30000 --res --snake --dual" "--cin 768 --cout 768 --k 1 --T 6000 --res --snake --dual"; do
      echo -n "rast$ra " >> $O/r.txt
      BC_X6_RASTER=$ra timeout -k 10 120 python tools/conv_bench.py $shp 2>&1 | grep "^Cin" >> $O/r.txt || exit 1
    done
    BC_X6_RASTER=$ra timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/b.json 2>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline']
print('rast$ra bench', d['value'], d['ms_per_step'], r['probe_bf16_tflops'], d['parity']['vs_reference_fixture']['index_mismatches'], [(k['kernel'][:44], k['ms_per_step']) for k in r['kernels_top'][:3]])" >> $O/r.txt
  done
done
sed 's/ TFLOP.*//' $O/r.txt
echo done
