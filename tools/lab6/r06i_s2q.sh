#!/bin/bash
# round 6: the phase-decomposed stride-2 convs on 16-byte sample-quad staging (conv1d_x6s2_kernel):
# its bit-identity / oracle tests, the two x6 stride-2 launches against BC_X6_S2Q=0 (single-float staging), same box
set -u
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "tiles_8_vs_16 or test_conv1d or k7_tiles" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do
  for q in 0 1; do
    for shp in "--cin 96 --cout 192 --k 4 --s 2 --T 60000 --snake" "--cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake"; do
      BC_X6_S2Q=$q timeout -k 10 100 python tools/conv_bench.py $shp --iters 10 2>&1 | grep Cin | sed "s/^/s2q=$q /" | tee -a $O/s2.txt
    done
  done
done
echo done
