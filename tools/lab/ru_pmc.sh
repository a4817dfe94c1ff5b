#!/bin/bash
# SQ / traffic counters of one ResidualUnit launch shape (tools/ru_bench.py), one counter group per rocprofv3 pass:
#   RU_ARGS="--C 48 --d 3 --T 240000 --lazy" bash tools/lab/ru_pmc.sh
set -u
R=${RPMC_DIR:-gpurun_out/rpmc}
mkdir -p $R
export TMPDIR=/tmp
ARGS=${RU_ARGS:---C 48 --d 3 --T 240000 --lazy}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA"
i=0
for ctr in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $R/p$i -o run -- \
    python3 tools/ru_bench.py --precision ${RU_PREC:-h3} --iters 3 $ARGS > $R/p$i.log 2>&1
  rc=$?; echo "[pass $i] exit $rc" >> $R/status.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
