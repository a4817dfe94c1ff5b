# Resampler timing at three rate pairs + the rocprofv3 kernel stats of the 16 -> 24 kHz run
set -u
mkdir -p gpurun_out/rsprof
export TMPDIR=/tmp
for r in "16000 24000" "44100 24000" "22050 24000"; do
  set -- $r
  timeout -k 10 120 python tools/resample_bench.py --orig $1 --new $2 >> gpurun_out/resample.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rsprof -o rs -- python3 tools/resample_bench.py > gpurun_out/rsprof.log 2>&1
