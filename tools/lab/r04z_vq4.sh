#!/bin/bash
# Round 4: the VQ forward with four lanes per frame (vq_fwd4_kernel) -- bit-identity tests, then config 2 A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04zv
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "vq or VQ or model or full or ops or fsq or rvq or config" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "FAIL|Error|assert" $O/tests.txt | head -20; exit 1; }
tail -1 $O/tests.txt
for v in 4 1 4 1; do
  BC_VQ_LANES=$v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-x6 > $O/c2_$v.json 2> $O/c2_$v.err || { echo "c2 failed $?"; exit 1; }
  python -c "import json;d=json.loads(open('$O/c2_$v.json').read().strip().splitlines()[-1]);print('lanes=$v', d['value'], d['ms_per_step'], d['parity']['vs_reference_fixture']['index_mismatches'])" >> $O/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-x6 --no-kernel-timer > $O/st.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
grep -h vq_fwd $O/st/run_kernel_stats.csv | cut -c1-200 >> $O/ab.txt
cat $O/ab.txt
