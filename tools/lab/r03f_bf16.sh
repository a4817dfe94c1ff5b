set -u
mkdir -p gpurun_out/r03f
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -v --timeout 120 --timeout-method thread -k "bf16 or reslstm or resunit_fused or lstm" > gpurun_out/r03f/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03f/tests.log; exit 1; }
tail -3 gpurun_out/r03f/tests.log
timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03f/bench5.json 2> gpurun_out/r03f/bench5.err || { echo "bench5 failed"; tail -20 gpurun_out/r03f/bench5.err; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-x6 > gpurun_out/r03f/bench2.json 2> gpurun_out/r03f/bench2.err || { echo "bench2 failed"; exit 1; }
python -c "
import json
for f in ['bench5','bench2']:
    d=json.loads(open('gpurun_out/r03f/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'], d.get('parity'), d['roofline']['kernel'], d['roofline']['frac'])
"
