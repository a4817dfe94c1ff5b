#!/bin/bash
# round 6: (1) where the x6 C = 48 / 96 one-launch units spend their time (BC_RU_DEBUG ablation bits on the
# BIGCODEC_ABLATION build under gpurun_abl/: 1 no A copies, 2 no B loads, 4 no epilogue, 8 no phase 2, 16 no Snake on
# load, 32 no phase-1 MFMAs, 64 no bridge Snake); (2) the k7 16-wave tile's counter traffic split:
# the same input through Cout = 768 (four 192-row m-groups re-staging it) and Cout = 192 (one), likewise at C = 384
set -u
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
# (0) the x6 ResLSTM with fp32 h hand-off: its tests, then the layer time against the session-start library (same box)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_streaming.py -k "lstm or reslstm or LSTM or stream or long30 or bidir" > $O/lstm_tests.txt 2>&1 || { echo "lstm tests failed"; tail -30 $O/lstm_tests.txt; exit 1; }
tail -1 $O/lstm_tests.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full_size.py > $O/full_tests.txt 2>&1 || { echo "full-size tests failed"; tail -30 $O/full_tests.txt; exit 1; }
tail -1 $O/full_tests.txt
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/base; else unset BIGCODEC_LIB_DIR; fi
    echo "$v $rep: $(timeout -k 10 120 python tools/lstm_bench.py --H 1536 --B 64 --T 1200 --precision x6 2>&1 | grep -v amdgpu.ids | tail -1)" | tee -a $O/lstm_ab.txt
  done
done
unset BIGCODEC_LIB_DIR
for C in 48 96; do
  T=$((240000 * 48 / C))
  for dbg in 0 1 2 4 8 16 32 64 127 0; do
    BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_RU_DEBUG=$dbg timeout -k 10 100 python tools/ru_bench.py --C $C --d 3 --T $T --precision x6 --lazy --iters 10 > $O/t.txt 2>&1 || { echo "ru failed"; tail $O/t.txt; exit 1; }
    echo "C=$C dbg $dbg: $(grep resunit $O/t.txt)" | tee -a $O/ru_abl.txt
  done
done
for shp in "--cin 768 --cout 768 --k 7 --d 1 --T 6000 --snake" "--cin 768 --cout 192 --k 7 --d 1 --T 6000 --snake" \
           "--cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake" "--cin 384 --cout 192 --k 7 --d 3 --T 30000 --snake"; do
  tag=$(echo $shp | awk '{print $2"_"$4"_"$10}')
  timeout -k 10 100 python tools/conv_bench.py $shp --iters 5 >> $O/conv_time.txt 2>&1 || { echo "conv failed"; exit 1; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/pmc_${tag}_$ctr -o run -- \
      python3 tools/conv_bench.py $shp --iters 3 > $O/pmc_${tag}_$ctr.log 2>&1 || { echo "pmc failed $tag $ctr"; tail $O/pmc_${tag}_$ctr.log; exit 1; }
  done
done
grep -v amdgpu.ids $O/conv_time.txt
echo done
