# Pointwise conv path: GPU conv tests (all precisions) + timing of the encoder's k=1 shapes
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -x -q tests/test_gpu_kernels.py -m gpu -k "conv1d or h3_block or x6_error or bf16_prec or reslstm" > gpurun_out/pw_tests.log 2>&1 || { echo "tests failed"; exit 1; }
run() { timeout -k 10 150 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> gpurun_out/pw.log 2>&1; }
run --cin 384 --cout 384 --k 1 --T 30000 --res --dual --snake --cfg 314,301,315,309 || exit 1
run --cin 192 --cout 192 --k 1 --T 60000 --res --dual --snake --cfg 314,301,315,309 || exit 1
run --cin 768 --cout 768 --k 1 --T 6000 --res --dual --snake --cfg 314,301,315,321 || exit 1
run --cin 1536 --cout 6144 --k 1 --T 76800 --B 1 --cfg 314,321,300 || exit 1
