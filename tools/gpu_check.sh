#!/bin/bash
# One GPU-box session: build check, GPU parity tests, smoke, short bench.  Every GPU step has its
# own time limit; a fault / abort / timeout (exit >= 124 or signal) stops the script.
set -u
mkdir -p gpurun_out
stop_if_fatal() { local rc=$1; local what=$2; echo "[$what] exit $rc" >> gpurun_out/status.log;
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ] && [ "$rc" -ne 5 ]; then echo "fatal at $what ($rc)"; exit "$rc"; fi; }
# the library is built here (CPU container) and travels in-tree; only check that it loads
python -c "from audiotokenization_amd import _lib; _lib.load()" > gpurun_out/build.log 2>&1 || { echo load failed; exit 2; }
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest ${TESTS:-tests} -m gpu -q -rA ${PYTEST_EXTRA:-} > gpurun_out/gpu_tests.log 2>&1
stop_if_fatal $? pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
stop_if_fatal $? smoke
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  stop_if_fatal $? bench
fi
echo done
