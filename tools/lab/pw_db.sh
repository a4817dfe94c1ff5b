# Pointwise convs: double-buffered, phase-staggered B (default) vs single buffer (BC_X6_PW_DB=0).
set -u
mkdir -p gpurun_out
out=gpurun_out/pw_db.log
: > $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_ops.py -m gpu \
  > gpurun_out/pw_db_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/pw_db_tests.log; exit 1; }
for db in 1 0 1 0; do
  echo "== PW_DB $db" >> $out
  run() { BC_X6_PW_DB=$db timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> $out 2>&1; }
  run --cin 192 --cout 192 --k 1 --T 60000 --res --dual || exit 1
  run --cin 384 --cout 384 --k 1 --T 30000 --res --dual || exit 1
  run --cin 768 --cout 768 --k 1 --T 6000 --res --dual || exit 1
  run --cin 1536 --cout 6144 --k 1 --T 1200 || exit 1
done
grep -v amdgpu.ids $out
