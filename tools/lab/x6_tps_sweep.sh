# Taps-per-K-step (BC_X6_TPS) x MFMA priority (BC_X6_DEBUG=16) sweep of the multi-tap h3 conv shapes.
set -u
mkdir -p gpurun_out
out=gpurun_out/tps.log
BC_X6_TPS=2 timeout -k 10 300 python -m pytest -x -q tests/test_gpu_kernels.py -m gpu -k "conv1d or h3_block or convT" > gpurun_out/tps_tests.log 2>&1 || { echo "tps2 tests failed"; exit 1; }
for tps in 1 2; do
  for dbg in 0 16; do
    echo "== TPS $tps dbg $dbg" >> $out
    run() { BC_X6_TPS=$tps BC_X6_DEBUG=$dbg timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> $out 2>&1; }
    run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake --cfg 309,300,314,315 || exit 1
    run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake --cfg 300,318,309 || exit 1
    run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake --cfg 309,315 || exit 1
    run --cin 1536 --cout 1024 --k 3 --T 1200 || exit 1
  done
done
