#!/bin/bash
# round 6: the whole GPU suite on the tree with the C = 192 one-launch unit, the strip-kernel offset fix and the
# library launch timer; smoke; the x6 bench line (kernels_top now with the ResLSTM / VQ launches)
set -u
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed"; tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; tail $O/smoke.txt; exit 1; }
grep smoke $O/smoke.txt
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench.json 2>$O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench', d['value'], d['ms_per_step'], r['probe_bf16_tflops'], d['parity']['vs_reference_fixture']['index_mismatches'], 'h3', d['h3']['value'])
print('timed total', r['all_timed_kernels_ms_per_step'], 'conv', r['all_python_conv_kernels_ms_per_step'])
for k in r['kernels_top']: print('   ', k['kernel'][:60], k['bound'], k['launches_per_step'], k['ms_per_step'], k['frac_mfma_spec'], k['frac_hbm'])"
echo done
