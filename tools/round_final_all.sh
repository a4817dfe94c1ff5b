#!/bin/bash
# End-of-session regression on ONE box: smoke, every -m gpu test, the default bench line, its rocprofv3
# kernel stats, configs 3-6, the PMC traffic passes.  Every GPU step has its own time limit; the first
# failure ends the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/final gpurun_out/stats
bash tools/round_final_a.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats -o run -- \
  python3 bench.py --no-cpu-baseline --no-x6 > gpurun_out/stats/bench.log 2>&1 || { echo "stats run failed $?"; exit 1; }
for c in 3 4 5 6; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-x6 > gpurun_out/final/bench_config$c.json 2> gpurun_out/final/bench_config$c.err || { echo "config $c failed $?"; exit 1; }
done
PMC_TIMEOUT=300 bash tools/gpu_pmc.sh || { echo "pmc failed $?"; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/final/bench_config2.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], d['parity']['vs_reference_fixture']['index_mismatches'], d['x6']['value'])"
grep -m1 "conv1d_x6_kernel<6, 2, 2, 8, 2, false, 2, false, true>" gpurun_out/stats/run_kernel_stats.csv
echo done
