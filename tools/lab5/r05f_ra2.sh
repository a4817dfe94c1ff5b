#!/bin/bash
# register-A x6 conv after the per-step weight resource: the shape that faulted first (alone), then the tile tests
set -u
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 60 python tools/lab5/ra_debug2.py > $O/ra_phase.txt 2>&1 || { echo "ra phase failed $?"; grep -v amdgpu.ids $O/ra_phase.txt | tail -5; exit 1; }
grep -v amdgpu.ids $O/ra_phase.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "tiles_8_vs_16 and x6 or k7_tiles_large or (test_conv1d and x6) or (narrow and x6)" --timeout 200 --timeout-method thread > $O/tests.txt 2>&1 || { echo "tests failed $?"; grep -E "^E |FAILED|passed|failed" $O/tests.txt | tail -20; exit 1; }
tail -2 $O/tests.txt
echo done
