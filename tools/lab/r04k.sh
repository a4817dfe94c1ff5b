#!/bin/bash
# Static priority for waves 8-15 of the 16-wave tile (BC_X6_PRIO=0 / 1, same box), the x6 pointwise launches on
# their pointwise B4 kernel, conv parity tests, bench config 2.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_full_size.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -2 $O/gpu_tests.txt; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; exit 1; }
for pr in 0 1 0 1; do
  for p in h3 x6 bf16; do
    for shape in "--cin 384 --cout 384 --k 7 --d 3 --T 30000 --snake" "--cin 768 --cout 768 --k 7 --d 3 --T 6000 --snake" "--cin 384 --cout 768 --k 10 --s 5 --T 6000 --snake"; do
      BC_X6_PRIO=$pr timeout -k 10 120 python tools/conv_bench.py --iters 5 --precision $p $shape >> $O/prio_$pr.txt 2>&1 || exit 1
    done
  done
done
paste <(grep Cin $O/prio_0.txt | sed 's/conv1d_x6_kernel//' | awk '{print $1,$2,$3,$4,$7,$(NF-5)}') <(grep Cin $O/prio_1.txt | awk '{print $(NF-5)}')
for shape in "--cin 192 --cout 192 --k 1 --T 60000 --res --dual" "--cin 384 --cout 384 --k 1 --T 30000 --res --dual" "--cin 768 --cout 768 --k 1 --T 6000 --res --dual"; do
  timeout -k 10 120 python tools/conv_bench.py --iters 10 --precision x6 $shape >> $O/x6_pw.txt 2>&1 || exit 1
done
grep Cin $O/x6_pw.txt | sed 's/conv1d_x6_kernel//'
timeout -k 10 500 python bench.py --no-cpu-baseline > $O/bench_config2.json 2> $O/bench_config2.err || { echo "bench failed $?"; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r04k/bench_config2.json").read().strip().splitlines()[-1])
r = d["roofline"]; x = d["x6"]
print(d["value"], r["kernel"], r["avg_launch_ms"], r["frac"], "x6", x["value"], x["roofline"]["frac"])
for row in x["roofline"]["kernels_top"][:3]: print(" x6", row["kernel"], row["launches_per_step"], row["ms_per_step"])
PY
echo done
