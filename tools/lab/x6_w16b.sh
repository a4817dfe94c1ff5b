# Historical (profiles/r02g_w16*.txt): cfg 322 / 323 / 324 here are the tile table of commit 3dcd5a4; only the
# 96 x 32-per-wave 16-wave tile was kept, and it is cfg 322 now (kX6Tiles index 22).
# 16-wave tiles, round 2: correctness of every 8- vs 16-wave pair, per-shape timing of the remaining
# tile classes, the A-prefetch on / off question for tile 123 (exp/noapf.so: the same tree built with
# APF off for 16-wave tiles), and the config-2 step under each BC_X6_W16 mask.
set -u
mkdir -p gpurun_out
out=gpurun_out/w16b.log
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu \
  -k "tiles_8_vs_16 or test_conv1d" > gpurun_out/w16b_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/w16b_tests.log; exit 1; }
tail -2 gpurun_out/w16b_tests.log
run() { timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 "$@" >> $out 2>&1; }
run --cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake --cfg 321,324 || exit 1
run --cin 1536 --cout 1024 --k 3 --d 1 --T 1200 --cfg 321,324 || exit 1
run --cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake --cfg 5320,5323 || exit 1
run --cin 768 --cout 1536 --k 10 --s 5 --T 1200 --cfg 5320,5323,5321,5324 || exit 1
run --cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake --cfg 2320,2323 || exit 1
run --cin 192 --cout 192 --k 1 --T 60000 --res --snake --dual --cfg 314,323 || exit 1
run --cin 384 --cout 384 --k 1 --T 30000 --res --snake --dual --cfg 314,323 || exit 1
run --cin 768 --cout 768 --k 1 --T 6000 --res --snake --dual --cfg 314,323 || exit 1
run --cin 1536 --cout 6144 --k 1 --T 76800 --B 1 --cfg 321,324 || exit 1
if [ -f exp/noapf.so ]; then
  cp audiotokenization_amd/libbigcodec_hip.so exp/main.so
  for lib in noapf main noapf main; do
    cp exp/$lib.so audiotokenization_amd/libbigcodec_hip.so
    echo "== $lib" >> $out
    run --cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake --cfg 320,323 || exit 1
    run --cin 384 --cout 384 --k 7 --d 9 --T 30000 --snake --cfg 320,323 || exit 1
  done
  cp exp/main.so audiotokenization_amd/libbigcodec_hip.so
fi
grep -v amdgpu.ids $out
for w in 1 3 7 15; do
  BC_X6_W16=$w timeout -k 10 300 python bench.py --no-cpu-baseline --no-x6 --steps 3 > gpurun_out/w16b_bench_$w.json 2> gpurun_out/w16b_bench_$w.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/w16b_bench_$w.json').read().strip().splitlines()[-1]); print('W16=$w', d['value'], d['ms_per_step'], d['parity']['vs_reference_fixture']['index_mismatches'])"
done
