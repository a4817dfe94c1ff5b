#!/bin/bash
# x6pw (pointwise double-buffered x6 tile): bit identity vs the 16-wave tile, then timing against it (BC_X6_PWDB=0)
set -u
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "pointwise_double or b4_staging or narrow_launch_tile" --timeout 100 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED|passed|failed" $O/tests.txt | tail; exit 1; }
tail -1 $O/tests.txt
for pw in 0 1; do
  for shp in "--cin 192 --cout 192 --T 60000" "--cin 384 --cout 384 --T 30000" "--cin 768 --cout 768 --T 6000"; do
    BC_X6_PWDB=$pw timeout -k 10 120 python tools/conv_bench.py $shp --k 1 --res --snake --dual >> $O/conv_pw$pw.txt 2>&1 || { echo "conv bench failed $?"; tail $O/conv_pw$pw.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/conv_pw0.txt $O/conv_pw1.txt
echo done
