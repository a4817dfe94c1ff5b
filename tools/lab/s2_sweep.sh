# Every h3 tile (direct and phase-decomposed) on the encoder's strided downsampling convs (dual output:
# raw for the next residual + SnakeBeta for the next conv).
set -u
mkdir -p gpurun_out
out=gpurun_out/s2.log
: > $out
run() { timeout -k 10 200 python tools/conv_bench.py --precision h3 --iters 5 --cfg all --dual "$@" >> $out 2>&1; }
run --cin 48 --cout 96 --k 4 --s 2 --T 120000 || exit 1
run --cin 96 --cout 192 --k 4 --s 2 --T 60000 || exit 1
run --cin 192 --cout 384 --k 4 --s 2 --T 30000 || exit 1
run --cin 384 --cout 768 --k 10 --s 5 --T 6000 || exit 1
run --cin 768 --cout 1536 --k 10 --s 5 --T 1200 || exit 1
grep -v amdgpu.ids $out
