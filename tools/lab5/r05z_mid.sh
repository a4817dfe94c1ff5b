#!/bin/bash
# x6 k7 (B4, one tap per K-step): the next step's copy issued after the first m-tile of MFMAs (current) against the
# copy issued at the step's start (gpurun_ab/head), alternating on one box; then the k7 tile parity tests
set -u
export TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
for rep in 1 2; do
  for v in head cur; do
    if [ $v = head ]; then export BIGCODEC_LIB_DIR=$PWD/gpurun_ab/head; else unset BIGCODEC_LIB_DIR; fi
    for shp in "--cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake" "--cin 384 --cout 384 --k 7 --d 9 --T 30000 --snake" "--cin 768 --cout 768 --k 7 --d 1 --T 6000 --snake"; do
      echo -n "$v " >> $O/m.txt
      timeout -k 10 120 python tools/conv_bench.py $shp 2>&1 | grep "^Cin" >> $O/m.txt || exit 1
    done
    timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/b.json 2>$O/b.err || { echo "bench failed"; tail $O/b.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v bench', d['value'], d['ms_per_step'], r['probe_bf16_tflops'], r['kernels_top'][0]['ms_per_step'])" >> $O/m.txt
  done
done
unset BIGCODEC_LIB_DIR
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_full_size.py -x -q -k "k7_tiles or conv1d or b4_staging or narrow or full_size" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED" $O/tests.txt | head; exit 1; }
tail -1 $O/tests.txt
cat $O/m.txt
echo done
