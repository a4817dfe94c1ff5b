# Double-buffered B tile (BC_X6_DB) A/B on the encoder's k7 h3 shapes, after the conv parity tests.
set -u
mkdir -p gpurun_out
out=gpurun_out/db.log
: > $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu \
  -k "conv1d or h3_block or convT or resunit" > gpurun_out/db_tests.log 2>&1 || { echo "db tests failed"; exit 1; }
for db in 0 1; do
  echo "== DB $db" >> $out
  run() { BC_X6_DB=$db timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> $out 2>&1; }
  for d in 1 3 9; do
    run --cin 192 --cout 192 --k 7 --d $d --T 60000 --snake || exit 1
    run --cin 384 --cout 384 --k 7 --d $d --T 30000 --snake || exit 1
    run --cin 768 --cout 768 --k 7 --d $d --T 6000 --snake || exit 1
  done
  run --cin 1536 --cout 1024 --k 3 --T 1200 || exit 1
  run --cin 96 --cout 96 --k 7 --d 3 --T 120000 --snake || exit 1
done
cat $out
