# Spread / staggered A copies (default) vs the burst after the barrier (BC_X6_DEBUG=64), k7 h3 shapes.
set -u
mkdir -p gpurun_out
out=gpurun_out/spread.log
: > $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu \
  > gpurun_out/spread_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/spread_tests.log; exit 1; }
for dbg in 0 64 0 64; do
  echo "== dbg $dbg" >> $out
  run() { BC_X6_DEBUG=$dbg timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> $out 2>&1; }
  run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake || exit 1
  run --cin 384 --cout 384 --k 7 --d 9 --T 30000 --snake || exit 1
  run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake || exit 1
  run --cin 384 --cout 768 --k 10 --s 5 --T 6000 --dual || exit 1
done
grep -v amdgpu.ids $out
