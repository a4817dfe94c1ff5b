# Every h3 tile on the encoder's pointwise (residual + dual output) convs.
set -u
mkdir -p gpurun_out
out=gpurun_out/pw_tiles.log
: > $out
run() { timeout -k 10 200 python tools/conv_bench.py --precision h3 --iters 5 --cfg all "$@" >> $out 2>&1; }
run --cin 192 --cout 192 --k 1 --T 60000 --res --dual || exit 1
run --cin 384 --cout 384 --k 1 --T 30000 --res --dual || exit 1
run --cin 768 --cout 768 --k 1 --T 6000 --res --dual || exit 1
grep -v amdgpu.ids $out
