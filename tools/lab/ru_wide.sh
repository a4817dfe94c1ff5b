# One-launch ResidualUnit with 256-column tiles (one workgroup per CU) vs the default 128-column ones
set -u
mkdir -p gpurun_out
for c in 0 106 104 105; do
  for shape in "--C 48 --d 1 --T 240000 --dual" "--C 96 --d 3 --T 120000 --dual"; do
    BC_RU_CFG=$c timeout -k 10 120 python tools/ru_bench.py $shape >> gpurun_out/ru_wide.log 2>&1 || echo "cfg $c failed for $shape" >> gpurun_out/ru_wide.log
  done
done
