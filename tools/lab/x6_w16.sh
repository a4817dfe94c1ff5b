# Historical (profiles/r02g_w16*.txt): cfg 322 / 323 / 324 here are the tile table of commit 3dcd5a4; only the
# 96 x 32-per-wave 16-wave tile was kept, and it is cfg 322 now (kX6Tiles index 22).
# 192 x 256 k7 tile: 8 waves (cfg 320) vs 16 waves (322: 48 x 64 per wave, 323: 96 x 32 per wave), h3.
set -u
mkdir -p gpurun_out
out=gpurun_out/w16.log
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu \
  -k "tiles_8_vs_16 or test_conv1d" > gpurun_out/w16_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/w16_tests.log; exit 1; }
for rep in 1 2; do
  run() { timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 --cfg 320,322,323 "$@" >> $out 2>&1; }
  run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake || exit 1
  run --cin 384 --cout 384 --k 7 --d 9 --T 30000 --snake || exit 1
done
grep -v amdgpu.ids $out
for w in 0 1 2; do
  BC_X6_W16=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 > gpurun_out/w16_bench_$w.json 2> gpurun_out/w16_bench_$w.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/w16_bench_$w.json').read().strip().splitlines()[-1]); print('W16=$w', d['value'], d['ms_per_step'], d['parity']['vs_reference_fixture']['index_mismatches'])"
done
