#!/bin/bash
# Round 3: per-launch layer profile of config 2 (h3) and config 5 (bf16, 32 x 30 s) on the current tree, and the
# kernel tests of the one-launch units (tile 123 now the h3 / bf16 default at C = 96).
set -u
mkdir -p gpurun_out
o=gpurun_out/r03o_layers.txt; : > $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "resunit" -x -q --timeout 120 --timeout-method thread >> $o 2>&1 || { echo "tests failed $?" >> $o; exit 1; }
timeout -k 10 200 python tools/layer_profile.py --precision h3 >> $o 2>&1 || { echo "layers h3 failed" >> $o; exit 1; }
timeout -k 10 200 python tools/layer_profile.py --precision bf16 --batch 32 --seconds 30 >> $o 2>&1 || { echo "layers bf16 failed" >> $o; exit 1; }
echo done >> $o
