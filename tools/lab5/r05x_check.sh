#!/bin/bash
# after the strided-tile selection change: model parity at full size, the conv tile tests, the x6 bench line
set -u
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_kernels.py -x -q -k "full_size or x6 or conv1d or k7_tiles or narrow" --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED" $O/tests.txt | head; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-h3 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], d['ms_per_step'], r['probe_bf16_tflops'], r['traffic'], d['parity']['vs_reference_fixture']['index_mismatches'], [(k['kernel'][:44], k['ms_per_step']) for k in r['kernels_top']])"
echo done
