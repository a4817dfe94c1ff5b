#!/bin/bash
# Round 4: adaptive strip length (C = 48 units) and the narrow rule on the 256 x 256 tile -- tests and stream timing.
set -u
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_streaming.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "narrow or stream or model or strip or c48 or resunit" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "FAIL|Error|assert" $O/tests.txt | head -20; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python tools/stream_bench.py --decode --B 16 --chunk 1000 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
timeout -k 10 300 python tools/stream_bench.py --chunk 4800 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
timeout -k 10 300 python tools/stream_bench.py --chunk 1200 --B 16 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-x6 > $O/c2.json 2> $O/c2.err || { echo "c2 failed $?"; exit 1; }
python -c "import json;d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]);print('config2', d['value'], d['ms_per_step'], d['parity'])" >> $O/stream.txt
grep -E "stream|config2" $O/stream.txt
