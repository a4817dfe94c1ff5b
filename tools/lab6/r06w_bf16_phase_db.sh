#!/bin/bash
# round 6: config 5's bf16 phase-decomposed strided convs (K / s = 2 taps per phase) on two taps per K-step with one B
# buffer (default) vs one tap per K-step over the double-buffered B tile (BC_X6_TPS=1), B = 32 x 30 s shapes
set -u
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
run() { timeout -k 10 120 python tools/conv_bench.py "$@" --B 32 --precision bf16 --iters 10 2>&1 | grep -v amdgpu.ids | tail -1 | sed 's/.*cfg=//'; }
for rep in 1 2; do
  for t in 2 1; do
    if [ $t = 1 ]; then export BC_X6_TPS=1; else unset BC_X6_TPS; fi
    echo "tps $t rep $rep | s2 96-192 $(run --cin 96 --cout 192 --k 4 --s 2 --T 180000 --snake) | s2 192-384 $(run --cin 192 --cout 384 --k 4 --s 2 --T 90000 --snake) | s5 384-768 $(run --cin 384 --cout 768 --k 10 --s 5 --T 18000 --snake) | s5 768-1536 $(run --cin 768 --cout 1536 --k 10 --s 5 --T 3600)" | tee -a $O/ab.txt
  done
done
echo done
