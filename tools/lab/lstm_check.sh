# ResLSTM: GPU tests + h3 stamp timeline + timing
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest -x -q tests/test_gpu_kernels.py -m gpu -k "reslstm" > gpurun_out/lstm_tests.log 2>&1 || { echo "tests failed"; exit 1; }
BC_LSTM_SEQ_STAMPS=1 timeout -k 10 120 python tools/lstm_bench.py --precision h3 > gpurun_out/lstm_stamps.log 2>&1 || exit 1
timeout -k 10 120 python tools/lstm_bench.py --precision h3 --layers 2 >> gpurun_out/lstm_stamps.log 2>&1 || exit 1
