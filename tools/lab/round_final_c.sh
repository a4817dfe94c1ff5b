#!/bin/bash
# Part A (smoke, every -m gpu test, the default bench line) plus two tile probes for the shapes still on
# the 256 x 256 tile (the LSTM input projection and the final k3).
set -u
bash tools/round_final_a.sh || exit 1
timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 --cin 1536 --cout 6144 --k 1 --T 76800 --B 1 --cfg 321,322 > gpurun_out/final/probe.log 2>&1 || exit 1
timeout -k 10 120 python tools/conv_bench.py --precision h3 --iters 5 --cin 1536 --cout 1024 --k 3 --T 1200 --cfg 321,322 >> gpurun_out/final/probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/final/probe.log
python -c "import json; d=json.loads(open('gpurun_out/final/bench_config2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['parity']['vs_reference_fixture']['index_mismatches'], d['x6']['value'])"
