#!/bin/bash
# Round 4: the ResLSTM input projection below 32 column tiles on the plain cfg-322 launch instead of presplit_b +
# pw_presplit (one presplit workgroup per 256 columns walks all 48 chunks: ~220 us whatever N) -- tests and timing.
set -u
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_streaming.py -x -q --timeout 300 --timeout-method thread -k "lstm or stream" > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "FAIL|Error|assert" $O/tests.txt | head -20; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python tools/stream_bench.py --decode --B 16 --chunk 1000 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
timeout -k 10 300 python tools/stream_bench.py --chunk 4800 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
timeout -k 10 300 python tools/stream_bench.py --chunk 1200 --B 16 >> $O/stream.txt 2>&1 || { echo "stream failed $?"; exit 1; }
for b in 1 4; do
  timeout -k 10 300 python bench.py --batch $b --steps 10 --warmup 2 --no-cpu-baseline --no-x6 > $O/b$b.json 2> $O/b$b.err || { echo "b$b failed $?"; exit 1; }
  python -c "import json;d=json.loads(open('$O/b$b.json').read().strip().splitlines()[-1]);print('B=$b x 10 s', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/step')" >> $O/stream.txt
done
grep -E "stream|B=" $O/stream.txt
