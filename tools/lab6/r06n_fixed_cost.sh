#!/bin/bash
# round 6: per-workgroup fixed cost of the x6 16-wave conv tile (cfg 122): the same output tile count (Cout = 192,
# B = 64 x 60 000 columns, k7 d = 3, snake epilogue) over Cin = 32 .. 768 (K-steps per workgroup = 7 Cin / 32), then the
# same with the epilogue ablated (BIGCODEC_ABLATION build, BC_X6_DEBUG=8); and the pointwise (k1) tile likewise
set -u
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
for cin in 32 64 96 192 384 768; do
  echo "k7 cin $cin: $(timeout -k 10 120 python tools/conv_bench.py --cin $cin --cout 192 --k 7 --d 3 --T 60000 --B 64 --snake --cfg 122 --iters 5 2>&1 | grep -v amdgpu.ids | tail -1)" | tee -a $O/fixed.txt
  echo "k7 cin $cin no-epi: $(BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_X6_DEBUG=8 timeout -k 10 120 python tools/conv_bench.py --cin $cin --cout 192 --k 7 --d 3 --T 60000 --B 64 --snake --cfg 122 --iters 5 2>&1 | grep -v amdgpu.ids | tail -1)" | tee -a $O/fixed.txt
done
for cin in 64 192 384 768 1536; do
  echo "k1 cin $cin: $(timeout -k 10 120 python tools/conv_bench.py --cin $cin --cout 384 --k 1 --T 30000 --B 64 --res --dual --cfg 122 --iters 5 2>&1 | grep -v amdgpu.ids | tail -1)" | tee -a $O/fixed.txt
  echo "k1 cin $cin no-epi: $(BIGCODEC_PKG_ROOT=$PWD/gpurun_abl BC_X6_DEBUG=8 timeout -k 10 120 python tools/conv_bench.py --cin $cin --cout 384 --k 1 --T 30000 --B 64 --res --dual --cfg 122 --iters 5 2>&1 | grep -v amdgpu.ids | tail -1)" | tee -a $O/fixed.txt
done
echo done
