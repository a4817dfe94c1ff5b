#!/bin/bash
# Round 4: the VQ forward's in_proj with 16 z loads in flight and the search unrolled by 4 -- tests, timing.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04zw
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "vq or VQ or model or full or ops or fsq or rvq or config or lstm or presplit" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "FAIL|Error|assert" $O/tests.txt | head -20; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-x6 --no-kernel-timer > $O/st.log 2>&1 || { echo "rocprof failed $?"; exit 1; }
grep -h "vq_\|presplit_b\|conv1d_mfma" $O/st/run_kernel_stats.csv | cut -c1-160
grep -h '"metric"' $O/st.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['vs_reference_fixture']['index_mismatches'])"
