#!/bin/bash
# SQ stall breakdown of one conv shape (tools/conv_bench.py), one counter group per rocprofv3 pass:
#   CONV_ARGS="--cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake" bash tools/lab/conv_pmc.sh
set -u
D=${CPMC_DIR:-gpurun_out/cpmc}
mkdir -p $D
export TMPDIR=/tmp
ARGS=${CONV_ARGS:---cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"
i=0
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for ctr in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i + 1))
  [ $i -gt ${CPMC_NPASS:-4} ] && break
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $D/p$i -o run -- \
    python3 tools/conv_bench.py --precision ${CONV_PREC:-h3} --iters 3 $ARGS > $D/p$i.log 2>&1
  rc=$?; echo "[pass $i] exit $rc" >> $D/status.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
