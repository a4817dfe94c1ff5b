set -u
mkdir -p gpurun_out
rm -f gpurun_out/x6_sweep.log
bash tools/x6_table_sweep.sh || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tiles_8_vs_16" > gpurun_out/g1_tests.txt 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/g1_tests.txt; exit 1; }
tail -2 gpurun_out/g1_tests.txt
echo ok
