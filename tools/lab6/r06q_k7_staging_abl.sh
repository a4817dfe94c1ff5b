#!/bin/bash
# round 6: what the x6 k7 launches' B staging costs (BIGCODEC_ABLATION build under gpurun_abl/, BC_X6_DEBUG: 2 no B loads,
# 4 no B stores (split + LDS writes), 6 both, 1 no A copies), k7 C = 384 / 768 / 192, d = 3, B = 64
set -u
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
run() { timeout -k 10 120 python tools/conv_bench.py "$@" --iters 10 2>&1 | grep -v amdgpu.ids | tail -1 | sed 's/.*): //'; }
for rep in 1 2; do
  for dbg in 0 4 2 6 1; do
    export BC_X6_DEBUG=$dbg
    echo "dbg $dbg rep $rep | k7_384 $(BIGCODEC_PKG_ROOT=$PWD/gpurun_abl run --cin 384 --cout 384 --k 7 --d 3 --T 30000 --B 64 --snake) | k7_768 $(BIGCODEC_PKG_ROOT=$PWD/gpurun_abl run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --B 64 --snake) | k7_192 $(BIGCODEC_PKG_ROOT=$PWD/gpurun_abl run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --B 64 --snake --cfg 122)" | tee -a $O/abl.txt
  done
done
echo done
