# stride-2 downsampling convs: the library's tiles vs the phase-decomposed 16-wave tile (2322).
set -u
mkdir -p gpurun_out
out=gpurun_out/s2_w16.log
: > $out
for rep in 1 2; do
  timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 --cin 96 --cout 192 --k 4 --s 2 --T 60000 --cfg 315,2320,2322 >> $out 2>&1 || exit 1
  timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 --cin 48 --cout 96 --k 4 --s 2 --T 120000 --cfg 2309,2322 >> $out 2>&1 || exit 1
done
grep -v amdgpu.ids $out
