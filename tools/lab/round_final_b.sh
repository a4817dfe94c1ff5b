#!/bin/bash
# End-of-round regression, part B: configs 3-6, rocprofv3 kernel stats of config 2, PMC traffic passes.
set -u
mkdir -p gpurun_out/final gpurun_out/stats
export TMPDIR=/tmp
for c in 3 4 5 6; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-x6 > gpurun_out/final/bench_config$c.json 2> gpurun_out/final/bench_config$c.err || { echo "config $c failed $?"; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- \
  python3 bench.py --no-cpu-baseline --no-x6 > gpurun_out/stats/bench.log 2>&1 || { echo "stats run failed $?"; exit 1; }
PMC_TIMEOUT=300 bash tools/gpu_pmc.sh || { echo "pmc failed $?"; exit 1; }
echo done
