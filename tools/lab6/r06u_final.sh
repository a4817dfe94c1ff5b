#!/bin/bash
# round-6 final evidence on the final library: every -m gpu test, smoke, PMC passes (HBM traffic, MFMA busy) of the x6
# config-2 bench, rocprofv3 kernel stats of the x6 and h3 benches, the default bench line (CPU baseline incl.)
set -u
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed $?"; grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; tail -3 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed $?"; tail $O/smoke.txt; exit 1; }
grep smoke $O/smoke.txt
PMC_DIR=$O/pmc PMC_TIMEOUT=300 bash tools/gpu_pmc.sh || { echo "pmc failed $?"; exit 1; }
echo pmc ok
for p in x6 h3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$p -o run -- \
    python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-h3 --precision $p > $O/prof_$p.log 2>&1 || { echo "rocprof $p failed $?"; tail $O/prof_$p.log; exit 1; }
done
echo prof ok
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed $?"; tail $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; h=d['h3']; rr=h['roofline']
print('x6', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], r['probe_bf16_tflops'], d['parity']['vs_reference_fixture']['index_mismatches'])
print('h3', h['value'], h['ms_per_step'], rr['kernel'], rr['avg_launch_ms'], rr['frac'], h['parity']['index_mismatches'])
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])
"
timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline --no-h3 > $O/bench_config5.json 2> $O/bench_config5.err || { echo "config 5 failed $?"; tail $O/bench_config5.err; exit 1; }
tail -c 300 $O/bench_config5.json
echo done
