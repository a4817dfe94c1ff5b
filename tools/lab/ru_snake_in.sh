#!/bin/bash
# Snake-on-load ResidualUnit A/B: parity tests, then the headline bench with and without it.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k resunit tests/test_gpu_model.py tests/test_gpu_streaming.py \
  > gpurun_out/ru_snake_in_tests.log 2>&1 || { echo tests failed $?; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/ru_snake_in_on.log 2>&1 || { echo bench on failed; exit 1; }
BIGCODEC_RU_SNAKE_IN=0 timeout -k 10 300 python bench.py > gpurun_out/ru_snake_in_off.log 2>&1 || { echo bench off failed; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/ru_snake_in_on2.log 2>&1 || { echo bench on2 failed; exit 1; }
echo done
