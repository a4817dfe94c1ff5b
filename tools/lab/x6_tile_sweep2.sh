# Swizzled 64-B B pitch + two taps per step: GPU conv/resunit tests, then the wide-tile sweep.
set -u
mkdir -p gpurun_out
out=gpurun_out/sweep2.log
timeout -k 10 400 python -m pytest -x -q tests/test_gpu_kernels.py -m gpu > gpurun_out/sweep2_tests.log 2>&1 || { echo "tests failed"; exit 1; }
run() { timeout -k 10 150 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> $out 2>&1; }
run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake --cfg 309,300,314,318,320,321 || exit 1
run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake --cfg 300,318,320,321 || exit 1
run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake --cfg 309,314,320 || exit 1
run --cin 1536 --cout 1024 --k 3 --T 1200 --cfg 300,318,320,321 || exit 1
run --cin 384 --cout 384 --k 1 --T 30000 --res --dual --snake --cfg 314 || exit 1
run --cin 192 --cout 192 --k 1 --T 60000 --res --dual --snake --cfg 314 || exit 1
run --cin 1536 --cout 6144 --k 1 --T 76800 --B 1 --cfg 314 || exit 1
run --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake || exit 1
run --cin 96 --cout 192 --k 4 --s 2 --T 60000 --snake || exit 1
