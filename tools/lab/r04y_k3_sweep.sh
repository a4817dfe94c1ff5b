#!/bin/bash
# Round 4: tiles for the final k3 conv (1536 -> 1024) at narrow launches.
set -u
O=gpurun_out/r04y
mkdir -p $O
for a in "--T 6 --B 16" "--T 24 --B 64" "--T 120 --B 64"; do
  timeout -k 10 240 python tools/conv_bench.py --precision h3 --cin 1536 --cout 1024 --k 3 $a --cfg 321,312,313,310,317,303,301 --iters 20 >> $O/sweep.txt 2>&1 || { echo "failed $?"; tail -3 $O/sweep.txt; exit 1; }
done
cut -c1-140 $O/sweep.txt
