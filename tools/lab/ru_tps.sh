# One-launch ResidualUnit: taps per K-step (BC_RU_TPS) on the encoder's unit shapes
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -x -q tests/test_gpu_kernels.py -m gpu -k "resunit or conv1d" > gpurun_out/ru_tests.log 2>&1 || { echo "tests failed"; exit 1; }
for tps in 1 2 4; do
  for shape in "--C 48 --d 1 --T 240000 --dual" "--C 48 --d 9 --T 240000" "--C 96 --d 3 --T 120000 --dual" "--C 96 --d 9 --T 120000"; do
    BC_RU_TPS=$tps timeout -k 10 120 python tools/ru_bench.py $shape >> gpurun_out/ru_tps.log 2>&1 || exit 1
  done
done
BC_LSTM_SEQ_STAMPS=1 timeout -k 10 120 python tools/lstm_bench.py --precision h3 > gpurun_out/lstm_stamps.log 2>&1 || exit 1
