# Ablation of the one-launch ResidualUnit (BC_RU_DEBUG bits, timing only): profiles/r01g_ru_ablation.txt
# needs a library built with BIGCODEC_ABLATION=1 (python audiotokenization_amd/build_lib.py): the product build compiles the switches out
set -u
mkdir -p gpurun_out
for dbg in 0 1 2 4 8 3 15; do
  BC_RU_DEBUG=$dbg timeout -k 10 120 python tools/ru_bench.py --C 48 --d 1 --T 240000 --dual >> gpurun_out/ru_abl.log 2>&1 || exit 1
  BC_RU_DEBUG=$dbg timeout -k 10 120 python tools/ru_bench.py --C 96 --d 3 --T 120000 --dual >> gpurun_out/ru_abl.log 2>&1 || exit 1
done
