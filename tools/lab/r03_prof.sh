#!/bin/bash
# Round 3 profile set: rocprofv3 kernel stats of the config-2 bench; SQ counters of the pointwise C = 384 conv and
# of the C = 96 ResidualUnit.  One rocprofv3 pass per counter group; the first failure ends it.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r03prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03prof/stats -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-x6 > gpurun_out/r03prof/bench.log 2>&1 || { echo "stats failed $?"; exit 1; }
CONV_ARGS="--cin 384 --cout 384 --k 1 --T 30000 --res --dual" bash tools/lab/conv_pmc.sh || { echo "conv pmc failed"; exit 1; }
RU_ARGS="--C 96 --d 3 --T 120000 --lazy" bash tools/lab/ru_pmc.sh || { echo "ru pmc failed"; exit 1; }
echo done
