# Every h3 tile on the ResLSTM input projection (k1 1536 -> 6144 over T = 1200) and the final k3 conv.
set -u
mkdir -p gpurun_out
out=gpurun_out/proj_tiles.log
: > $out
run() { timeout -k 10 200 python tools/conv_bench.py --precision h3 --iters 5 --cfg all "$@" >> $out 2>&1; }
run --cin 1536 --cout 6144 --k 1 --T 1200 || exit 1
run --cin 1536 --cout 1024 --k 3 --T 1200 || exit 1
grep -v amdgpu.ids $out
