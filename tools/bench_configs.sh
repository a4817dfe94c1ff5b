# bench.py configs 3 / 4 / 5 (config 2 is the default run) -> gpurun_out/bench_c*.log
set -u
mkdir -p gpurun_out
for c in 3 4 5; do
  timeout -k 10 600 python bench.py --config $c > gpurun_out/bench_c$c.log 2>&1 || { echo "config $c failed"; exit 1; }
done
