#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (profiles/ summaries are copied from here).
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
  python3 bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline} > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "[rocprof] exit $rc" >> gpurun_out/status.log; exit $rc
