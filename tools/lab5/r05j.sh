#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
run() { timeout -k 10 120 python tools/conv_bench.py "$@" >> $O/conv.txt 2>&1 || { echo "conv bench failed $?"; tail $O/conv.txt; exit 1; }; }
run --cin 384 --cout 384 --k 1 --T 30000 --res --snake --dual --cfg 122,120
run --cin 192 --cout 192 --k 1 --T 60000 --res --snake --dual --cfg 122,120
run --cin 768 --cout 768 --k 1 --T 6000 --res --snake --dual --cfg 122,120
grep -v amdgpu.ids $O/conv.txt
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "tiles_8_vs_16 and x6" --timeout 100 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED|passed|failed" $O/tests.txt | tail; exit 1; }
tail -1 $O/tests.txt
echo done
