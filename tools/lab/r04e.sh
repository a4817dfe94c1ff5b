#!/bin/bash
# ResidualUnit C = 96 (cfg 323, h3, snake on load, d = 3) work-skipping ablation on the BIGCODEC_ABLATION build under
# gpurun_abl/ (BC_RU_DEBUG bits: 1 A copies, 2 B loads, 4 epilogue, 8 phase 2, 16 Snake on load, 32 phase-1 MFMAs,
# 64 bridge Snake; timing only, wrong results), then SQ / traffic counters of the product C = 96 unit and C = 48 strip.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
for dbg in 0 1 2 4 8 16 32 64 3 12 80 127; do
  echo "== dbg $dbg" >> $O/ru_ablation.txt
  BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_RU_DEBUG=$dbg timeout -k 10 120 python tools/ru_bench.py --C 96 --d 3 --T 120000 --lazy --cfg 323 --iters 5 >> $O/ru_ablation.txt 2>&1 || exit 1
done
grep -E "==|resunit" $O/ru_ablation.txt
RPMC_DIR=$O/pmc96 RU_ARGS="--C 96 --d 3 --T 120000 --lazy --cfg 323" bash tools/lab/ru_pmc.sh || { echo "pmc 96 failed"; exit 1; }
RPMC_DIR=$O/pmc48 RU_ARGS="--C 48 --d 3 --T 240000 --lazy" bash tools/lab/ru_pmc.sh || { echo "pmc 48 failed"; exit 1; }
python tools/pmc_dump.py $O/pmc96 resunit > $O/pmc96.txt
python tools/pmc_dump.py $O/pmc48 resunit > $O/pmc48.txt
rm -rf $O/pmc96/p* $O/pmc48/p*
cat $O/pmc96.txt $O/pmc48.txt
echo done
