#!/bin/bash
# Fused epilogue of the 16-wave tile (FE): conv parity tests, same-box A/B (BC_X6_FE=0 / 1) on the encoder's k7 and
# strided shapes in h3 / x6 / bf16, bench config 2 and 5.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; exit 1; }
for fe in 0 1; do
  for p in h3 x6 bf16; do
    for shape in "--cin 192 --cout 192 --k 7 --d 3 --T 60000 --snake" "--cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake" "--cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake" "--cin 192 --cout 384 --k 4 --s 2 --T 30000 --snake" "--cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake"; do
      BC_X6_FE=$fe timeout -k 10 120 python tools/conv_bench.py --iters 5 --precision $p $shape >> $O/fe_ab_$fe.txt 2>&1 || exit 1
    done
  done
done
paste <(grep Cin $O/fe_ab_0.txt | sed 's/conv1d_x6_kernel//' | awk '{print $1,$2,$3,$4,$5,$7,$(NF-5)}') <(grep Cin $O/fe_ab_1.txt | awk '{print $(NF-5)}')
timeout -k 10 500 python bench.py --no-cpu-baseline > $O/bench_config2.json 2> $O/bench_config2.err || { echo "bench failed $?"; exit 1; }
timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline > $O/bench_config5.json 2> $O/bench_config5.err || { echo "config 5 failed $?"; exit 1; }
python - <<'PY'
import json
for c in (2, 5):
    d = json.loads(open(f"gpurun_out/r04i/bench_config{c}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(c, d["value"], d["ms_per_step"], r["kernel"], r["avg_launch_ms"], r["frac"], d.get("x6", {}) and d["x6"]["value"])
    for row in r["kernels_top"][:4]: print(" ", row["kernel"], row["launches_per_step"], row["ms_per_step"], row["frac_mfma_spec"])
PY
echo done
