#!/bin/bash
# Round 4 pass: the ResidualUnit ablation + PMC (r04e), then the 16-byte pointwise staging: kernel tests (incl. the
# B4 / single-float bit-identity test), full-size tests, pointwise A/B (BC_X6_B4=0 vs 1) and the bench.
set -u
export TMPDIR=/tmp
bash tools/lab/r04e.sh || exit 1
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_full_size.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; exit 1; }
for b4 in 0 1; do
  for shape in "--cin 384 --cout 384 --k 1 --T 30000 --res --dual" "--cin 768 --cout 768 --k 1 --T 6000 --res --dual" "--cin 192 --cout 192 --k 1 --T 60000 --res --dual"; do
    for p in h3 x6 bf16; do
      BC_X6_B4=$b4 timeout -k 10 120 python tools/conv_bench.py --iters 10 --precision $p $shape >> $O/pw_b4_ab.txt 2>&1 || exit 1
    done
  done
done
grep -v amdgpu.ids $O/pw_b4_ab.txt
timeout -k 10 500 python bench.py --no-cpu-baseline > $O/bench_config2.json 2> $O/bench_config2.err || { echo "bench failed $?"; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r04f/bench_config2.json").read().strip().splitlines()[-1])
r = d["roofline"]; x = d["x6"]; rr = x["roofline"]
print(d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"])
print("x6", x["value"], x["ms_per_step"], rr["kernel"], rr["avg_launch_ms"], rr["frac"], x["parity"]["index_mismatches"])
for row in r["kernels_top"]: print(row["kernel"], row["launches_per_step"], row["ms_per_step"], row["frac_mfma_spec"], row["frac_hbm"])
PY
echo done
