#!/bin/bash
# rocprofv3 kernel-trace statistics of the default bench command, then the PMC passes (tools/gpu_pmc.sh).
set -u
mkdir -p gpurun_out/stats
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- \
  python3 bench.py > gpurun_out/stats/bench.log 2>&1 || { echo "stats run failed $?"; exit 1; }
bash tools/gpu_pmc.sh || { echo "pmc failed $?"; exit 1; }
echo done
