# One-launch ResidualUnit at three workgroups per CU (BC_RU_OCC=6, 80 VGPRs) vs two
set -u
mkdir -p gpurun_out
timeout -k 10 300 env BC_RU_OCC=6 python -m pytest -x -q tests/test_gpu_kernels.py -m gpu -k "resunit" > gpurun_out/ru_occ_tests.log 2>&1 || { echo "tests failed"; exit 1; }
for occ in 0 6; do
  for tps in 1 2 0; do
    for shape in "--C 48 --d 1 --T 240000 --dual" "--C 96 --d 3 --T 120000 --dual"; do
      BC_RU_OCC=$occ BC_RU_TPS=$tps timeout -k 10 120 python tools/ru_bench.py $shape >> gpurun_out/ru_occ.log 2>&1 || exit 1
      echo "   (occ=$occ tps=$tps)" >> gpurun_out/ru_occ.log
    done
  done
done
