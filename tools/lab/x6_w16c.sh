# Historical (profiles/r02g_w16*.txt): cfg 322 / 323 / 324 here are the tile table of commit 3dcd5a4; only the
# 96 x 32-per-wave 16-wave tile was kept, and it is cfg 322 now (kX6Tiles index 22).
# 16-wave tile 122: correctness (every 8- vs 16-wave pair, the conv cases) and the config-2 step under
# BC_X6_W16 masks 3 (default: k7 + strided), 7 (+ k7 C = 768), 11 (+ pointwise C = 192).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu \
  -k "tiles_8_vs_16 or test_conv1d" > gpurun_out/w16c_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/w16c_tests.log; exit 1; }
tail -1 gpurun_out/w16c_tests.log
timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake --cfg 321,322 > gpurun_out/w16c.log 2>&1 || exit 1
timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 --cin 192 --cout 192 --k 1 --T 60000 --res --snake --dual --cfg 314,322 >> gpurun_out/w16c.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/w16c.log
for w in 3 7 11 3; do
  BC_X6_W16=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 > gpurun_out/w16c_bench_$w.json 2> gpurun_out/w16c_bench_$w.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/w16c_bench_$w.json').read().strip().splitlines()[-1]); print('W16=$w', d['value'], d['ms_per_step'], d['parity']['vs_reference_fixture']['index_mismatches'])"
done
