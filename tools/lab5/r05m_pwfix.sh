#!/bin/bash
# pointwise 16-wave tile with the staging registers consumed before the A copy (no vmcnt(0) over fresh loads):
# timing vs the x6pw tile, then the pointwise / staging parity tests
set -u
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
for pw in 0 1; do
  for shp in "--cin 192 --cout 192 --T 60000" "--cin 384 --cout 384 --T 30000" "--cin 768 --cout 768 --T 6000"; do
    BC_X6_PWDB=$pw timeout -k 10 120 python tools/conv_bench.py $shp --k 1 --res --snake --dual >> $O/conv_pw$pw.txt 2>&1 || { echo "conv bench failed $?"; tail $O/conv_pw$pw.txt; exit 1; }
  done
done
for prec in h3 bf16; do
  for shp in "--cin 192 --cout 192 --T 60000" "--cin 384 --cout 384 --T 30000" "--cin 768 --cout 768 --T 6000"; do
    timeout -k 10 120 python tools/conv_bench.py $shp --k 1 --res --snake --dual --precision $prec >> $O/conv_$prec.txt 2>&1 || { echo "conv bench failed $?"; tail $O/conv_$prec.txt; exit 1; }
  done
done
grep -hv amdgpu.ids $O/conv_*.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "pointwise_double or b4_staging or narrow_launch_tile or presplit or test_conv1d" --timeout 100 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED|passed|failed" $O/tests.txt | tail; exit 1; }
tail -1 $O/tests.txt
echo done
