#!/bin/bash
# PMC passes (one counter group per pass, kernel-trace only — no sys/runtime trace):
#   FETCH_SIZE, WRITE_SIZE          -> HBM traffic per launch (tools/pmc_summary.py)
#   SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE -> MFMA utilisation per launch
set -u
D=${PMC_DIR:-gpurun_out/pmc}
mkdir -p $D
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timer --no-h3}
PASSES=${PMC_PASSES:-"FETCH_SIZE WRITE_SIZE MFMA"}
for pass in $PASSES; do
  ctr=$pass
  [ "$pass" = "MFMA" ] && ctr="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
  timeout -k 10 ${PMC_TIMEOUT:-600} rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $D/$pass -o run -- \
    python3 bench.py $ARGS > $D/$pass.log 2>&1
  rc=$?; echo "[pmc $pass] exit $rc" >> gpurun_out/status.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
