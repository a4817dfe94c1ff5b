#!/bin/bash
# round 6: does the XCD-aware workgroup remap (bc_common.h xcd_remap) put a k7 tile's 192-row m-group siblings on one
# XCD?  The m-group count multiplies the k7 input's fetched bytes (profiles/r06d_k7_traffic_split.json).  Same box:
# the product library (remap) against a build with BIGCODEC_NO_XCD_REMAP=1 (gpurun_abl/: the dispatcher's order),
# per-launch times, FETCH_SIZE of the C = 768 / 384 k7 launches, and the x6 bench line of both.
set -u
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
ABL=$PWD/gpurun_abl/audiotokenization_amd
for rep in 1 2; do
  for v in remap noremap; do
    if [ $v = noremap ]; then export BIGCODEC_LIB_DIR=$ABL; else unset BIGCODEC_LIB_DIR; fi
    for shp in "--cin 768 --cout 768 --k 7 --d 1 --T 6000 --snake" "--cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake" \
               "--cin 384 --cout 384 --k 1 --T 30000 --res --snake --dual" "--cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake"; do
      echo "$v: $(timeout -k 10 100 python tools/conv_bench.py $shp --iters 5 2>&1 | grep -v amdgpu.ids | tail -1)" | tee -a $O/times.txt
    done
  done
done
for v in remap noremap; do
  if [ $v = noremap ]; then export BIGCODEC_LIB_DIR=$ABL; else unset BIGCODEC_LIB_DIR; fi
  for shp in "--cin 768 --cout 768 --k 7 --d 1 --T 6000 --snake" "--cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake"; do
    tag=$(echo $shp | awk '{print $2"_"$4"_"$10}')
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_${v}_${tag} -o run -- \
      python3 tools/conv_bench.py $shp --iters 3 > $O/pmc_${v}_${tag}.log 2>&1 || { echo "pmc failed"; tail $O/pmc_${v}_${tag}.log; exit 1; }
  done
done
for v in remap noremap remap noremap; do
  if [ $v = noremap ]; then export BIGCODEC_LIB_DIR=$ABL; else unset BIGCODEC_LIB_DIR; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/bench_$v.json 2>$O/bench_$v.err || { echo "bench failed"; tail $O/bench_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench $v', d['value'], d['ms_per_step'], r['probe_bf16_tflops'], d['parity']['vs_reference_fixture']['index_mismatches'])
for k in r['kernels_top'][:9]: print('   ', k['kernel'][:50], k['launches_per_step'], k['ms_per_step'])" | tee -a $O/bench.txt
done
echo done
