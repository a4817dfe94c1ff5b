# Pointwise / residual-epilogue conv shapes of the encoder (h3, dual output), library choice.
set -u
mkdir -p gpurun_out
out=gpurun_out/pw.log
: > $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu \
  > gpurun_out/pw_tests.log 2>&1 || { echo "kernel tests failed"; tail -20 gpurun_out/pw_tests.log; exit 1; }
run() { timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> $out 2>&1; }
run --cin 192 --cout 192 --k 1 --T 60000 --res --dual || exit 1
run --cin 384 --cout 384 --k 1 --T 30000 --res --dual || exit 1
run --cin 768 --cout 768 --k 1 --T 6000 --res --dual || exit 1
run --cin 384 --cout 384 --k 1 --T 30000 --res || exit 1
timeout -k 10 100 python tools/ru_bench.py --C 96 --d 3 --T 120000 --dual > gpurun_out/pw_ru.log 2>&1 || exit 1
timeout -k 10 100 python tools/ru_bench.py --C 48 --d 3 --T 240000 --dual >> gpurun_out/pw_ru.log 2>&1 || exit 1
grep -v amdgpu.ids $out; grep -v amdgpu.ids gpurun_out/pw_ru.log | tail -12
