# Ablation of the conv kernel main loop (BC_X6_DEBUG bits: 1 no A copies, 2 no B loads, 4 no B stores, 8 no epilogue);
# needs a library built with BIGCODEC_ABLATION=1 (python audiotokenization_amd/build_lib.py): the product build compiles the switches out
# results in profiles/r01f_h3_x6kernel_ablation.txt.  Timing only: the outputs are wrong with any bit set.
set -u
mkdir -p gpurun_out
for dbg in 0 1 2 4 8 3 7 15; do
  echo "== dbg $dbg" >> gpurun_out/dbg.log
  BC_X6_DEBUG=$dbg timeout -k 10 120 python tools/conv_bench.py --precision h3 --cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake --cfg 309,300,318 --iters 5 >> gpurun_out/dbg.log 2>&1 || exit 1
  BC_X6_DEBUG=$dbg timeout -k 10 120 python tools/conv_bench.py --precision h3 --cin 384 --cout 384 --k 1 --T 30000 --res --dual --cfg 314 --iters 5 >> gpurun_out/dbg.log 2>&1 || exit 1
done
