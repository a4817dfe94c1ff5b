#!/bin/bash
# round 6: the one-launch units' h tile swizzled by (n >> 1) & 3 (conflict-free phase-2 fragment reads) -- unit tests,
# then the units and the x6 line against the previous library (gpurun_ab/prev), alternating on one box, and one PMC pass
set -u
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -rA --timeout 300 --timeout-method thread \
  -k "resunit or strip or w16" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
ru() { timeout -k 10 100 python tools/ru_bench.py "$@" --lazy --iters 10 2>&1 | grep resunit | sed 's/.*: //'; }
for rep in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/prev; else unset BIGCODEC_LIB_DIR; fi
    echo "$v $rep | x6 48 $(ru --C 48 --d 3 --T 240000 --precision x6) | x6 96 $(ru --C 96 --d 3 --T 120000 --precision x6) | x6 192 $(ru --C 192 --d 3 --T 60000 --precision x6) | h3 48 $(ru --C 48 --d 3 --T 240000 --precision h3)" | tee -a $O/ab.txt
  done
done
for v in prev new prev new; do
  if [ $v = prev ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/prev; else unset BIGCODEC_LIB_DIR; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/bench_$v.json 2>$O/bench_$v.err || { echo "bench failed"; tail $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench $v', d['value'], d['ms_per_step'], d['parity']['vs_reference_fixture']['index_mismatches'])
for k in r['kernels_top'][:8]: print('   %-58s %2d %8.3f' % (k['kernel'][:58], k['launches_per_step'], k['ms_per_step']))" | tee -a $O/ab.txt
done
unset BIGCODEC_LIB_DIR
CTR="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES"
for C in 48 96 192; do
  T=$((240000 * 48 / C))
  timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $O/pmc/ru$C -o run -- \
    python3 tools/ru_bench.py --C $C --d 3 --T $T --precision x6 --lazy --iters 3 > $O/ru$C.log 2>&1 || { echo "ru$C pmc failed $?"; tail -5 $O/ru$C.log; exit 1; }
done
python3 tools/pmc_dump.py $O/pmc resunit > $O/pmc_summary.txt
cat $O/pmc_summary.txt
echo done
