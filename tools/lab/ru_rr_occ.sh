# resunit_rr at C = 48: the shipped build (93 VGPRs, 5 waves per SIMD) vs exp/rr6.so (the same tree with
# __launch_bounds__(..., 6): <= 80 VGPRs, 6 waves per SIMD).
set -u
mkdir -p gpurun_out
out=gpurun_out/ru_rr_occ.log
: > $out
cp audiotokenization_amd/libbigcodec_hip.so exp/main.so
for lib in main rr6 main rr6; do
  cp exp/$lib.so audiotokenization_amd/libbigcodec_hip.so
  for d in 1 9; do
    echo "== $lib d=$d" >> $out
    timeout -k 10 120 python tools/ru_bench.py --C 48 --d $d --T 240000 --lazy --dual >> $out 2>&1 || exit 1
  done
done
cp exp/main.so audiotokenization_amd/libbigcodec_hip.so
grep -v amdgpu.ids $out
