#!/bin/bash
# the kernel / ops / model GPU tests on the bounds-checked debug build (every test also asserts no failed index check)
set -u
export TMPDIR=/tmp
O=${DBG_OUT:-gpurun_out/r05ze}
mkdir -p $O
BIGCODEC_DEBUG=1 timeout -k 10 1000 python -u -m pytest ${DBG_TESTS:-tests/test_gpu_kernels.py tests/test_gpu_ops.py tests/test_gpu_model.py} -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { echo "debug tests failed $?"; grep -E "^E |FAILED" $O/tests.txt | head -20; tail -3 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
echo done
