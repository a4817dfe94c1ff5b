#!/bin/bash
# PMC traffic passes (one counter group per pass, kernel-trace only — no sys/runtime trace).
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timer}
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 ${PMC_TIMEOUT:-600} rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d gpurun_out/pmc/$ctr -o run -- \
    python3 bench.py $ARGS > gpurun_out/pmc/$ctr.log 2>&1
  rc=$?; echo "[pmc $ctr] exit $rc" >> gpurun_out/status.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
