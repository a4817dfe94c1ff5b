#!/bin/bash
# round 6: LDS bank conflicts and instruction mix of the x6 k7 tile (C = 384) and the x6 C = 48 / 96 / 192 units (one
# rocprofv3 --pmc pass per program, 8 SQ counters, kernel trace only)
set -u
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
CTR="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $O/k7 -o run -- \
  python3 tools/conv_bench.py --cin 384 --cout 384 --k 7 --d 3 --T 30000 --B 64 --snake --iters 3 > $O/k7.log 2>&1 || { echo "k7 pmc failed $?"; tail -5 $O/k7.log; exit 1; }
for C in 48 96 192; do
  T=$((240000 * 48 / C))
  timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $O/ru$C -o run -- \
    python3 tools/ru_bench.py --C $C --d 3 --T $T --precision x6 --lazy --iters 3 > $O/ru$C.log 2>&1 || { echo "ru$C pmc failed $?"; tail -5 $O/ru$C.log; exit 1; }
done
python3 tools/pmc_dump.py $O > $O/summary.txt
cat $O/summary.txt
echo done
