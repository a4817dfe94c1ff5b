#!/bin/bash
# ResidualUnit coefficient prefetch (bridge passes, epilogue row coefficients, snake-on-load coefficients once):
# unit timings at encoder shapes (x6 / h3), then the unit and conv parity tests
set -u
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
for p in x6 h3; do
  for d in 1 3 9; do
    timeout -k 10 100 python tools/ru_bench.py --C 48 --d $d --T 240000 --precision $p --lazy --dual >> $O/ru.txt 2>&1 || { echo "ru bench failed $?"; tail $O/ru.txt; exit 1; }
    timeout -k 10 100 python tools/ru_bench.py --C 96 --d $d --T 120000 --precision $p --lazy --dual >> $O/ru.txt 2>&1 || { echo "ru bench failed $?"; tail $O/ru.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/ru.txt
for shp in "--cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake" "--cin 384 --cout 384 --T 30000 --k 1 --res --snake --dual" "--cin 768 --cout 768 --k 7 --d 9 --T 6000 --snake"; do
  timeout -k 10 120 python tools/conv_bench.py $shp >> $O/conv.txt 2>&1 || { echo "conv bench failed $?"; tail $O/conv.txt; exit 1; }
done
grep -v amdgpu.ids $O/conv.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "resunit or strip or conv1d or b4_staging or narrow or k7_tiles" --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED|passed|failed" $O/tests.txt | tail -20; exit 1; }
tail -1 $O/tests.txt
echo done
