#!/bin/bash
# static s_setprio(1) for the 16-wave tile's younger half (BC_X6_PRIO=1) on the x6 k7 / pointwise shapes, alternating
set -u
export TMPDIR=/tmp
O=gpurun_out/r05y
mkdir -p $O
for rep in 1 2; do
  for pr in 0 1; do
    for shp in "--cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake" "--cin 384 --cout 384 --k 7 --d 9 --T 30000 --snake" "--cin 768 --cout 768 --k 7 --d 1 --T 6000 --snake" "--cin 384 --cout 384 --k 1 --T 30000 --res --snake --dual"; do
      echo -n "prio$pr " >> $O/p.txt
      BC_X6_PRIO=$pr timeout -k 10 120 python tools/conv_bench.py $shp 2>&1 | grep "^Cin" >> $O/p.txt || exit 1
    done
  done
done
cat $O/p.txt
echo done
