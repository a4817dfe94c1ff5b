#!/bin/bash
# ResidualUnit input staging with 4 pairs x 8 columns per half-wave (gpurun_ab/new) against 1 pair x 32 columns (the
# tree's library), alternating on one box; the new build's bank-conflict counter; its unit parity tests
set -u
export TMPDIR=/tmp
O=gpurun_out/r05zi
mkdir -p $O
for rep in 1 2; do
  for v in head new; do
    if [ $v = new ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/new; else unset BIGCODEC_LIB_DIR; fi
    for a in "--C 48 --d 3 --T 240000 --precision x6" "--C 96 --d 3 --T 120000 --precision x6" "--C 96 --d 3 --T 120000 --precision h3" "--C 96 --d 9 --T 360000 --B 32 --precision bf16"; do
      echo -n "$v " >> $O/m.txt
      timeout -k 10 120 python tools/ru_bench.py $a --lazy --dual 2>&1 | grep "^resunit" >> $O/m.txt || exit 1
    done
  done
done
export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/new
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "resunit" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED" $O/tests.txt | head; exit 1; }
tail -1 $O/tests.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $O/pmc -o run -- python3 tools/ru_bench.py --C 48 --d 3 --T 240000 --precision x6 --lazy --dual --iters 3 > $O/pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $O/pmc96 -o run -- python3 tools/ru_bench.py --C 96 --d 3 --T 120000 --precision x6 --lazy --dual --iters 3 > $O/pmc96.log 2>&1 || { echo "pmc failed"; exit 1; }
sed 's/ TFLOP.*//' $O/m.txt
echo done
