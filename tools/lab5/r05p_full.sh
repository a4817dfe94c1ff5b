#!/bin/bash
# full GPU regression of the current tree: smoke, every -m gpu test, the default bench line (x6 headline + h3 leg),
# rocprof kernel stats of the x6 bench
set -u
export TMPDIR=/tmp
O=${FULL_OUT:-gpurun_out/r05p}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed $?"; tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { echo "gpu tests failed $?"; grep -E "^E |FAILED" $O/gpu_tests.txt | head -20; tail -3 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 500 python bench.py --steps 10 --warmup 2 --cpu-clips 1 --cpu-batches "" > $O/bench.json 2> $O/bench.err || { echo "bench failed $?"; tail $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; h=d['h3']; rr=h['roofline']
print('x6', d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], r['frac'], d['parity']['vs_reference_fixture']['index_mismatches'])
print('h3', h['value'], h['ms_per_step'], rr['kernel'], rr['avg_launch_ms'], rr['frac'], h['parity']['index_mismatches'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-h3 > $O/prof.log 2>&1 || { echo "rocprof failed $?"; tail $O/prof.log; exit 1; }
echo done
