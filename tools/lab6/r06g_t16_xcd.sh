#!/bin/bash
# round 6: (1) the x6 C = 48 unit's 16-channel tail on K16 MFMAs (resunit_x6_kernel<..., T16 = true>): its tests and
# unit times against BC_RU_T16=0 (the zero-padded K32 chunk), same box; (2) where the dispatcher puts the workgroups of a
# one-per-CU grid (HW_REG_XCC_ID per workgroup: tools/lab6/xcd_probe.hip)
set -u
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 60 ./tools/lab6/xcd_probe.bin 4096 1024 > $O/xcd_probe.txt 2>&1 || { echo "probe failed"; tail $O/xcd_probe.txt; exit 1; }
python3 - <<'PY'
rows=[l.split() for l in open('gpurun_out/r06g/xcd_probe.txt') if l[0].isdigit()]
x=[int(r[1]) for r in rows]
print('first 64 workgroups -> xcc:', ''.join(str(v) for v in x[:64]))
print('workgroups 256-319 -> xcc:', ''.join(str(v) for v in x[256:320]))
import collections
print('per-xcc counts:', sorted(collections.Counter(x).items()))
print('i % 8 == xcc for', sum(1 for i, v in enumerate(x) if i % 8 == v), 'of', len(x))
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_abi.py -k "resunit or abi or kernel_name" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_full_size.py tests/test_gpu_model.py > $O/tests2.txt 2>&1 || { echo "model tests failed"; tail -30 $O/tests2.txt; exit 1; }
tail -1 $O/tests2.txt
for rep in 1 2; do
  for t16 in 0 1; do
    for d in 1 9; do
      BC_RU_T16=$t16 timeout -k 10 100 python tools/ru_bench.py --C 48 --d $d --T 240000 --precision x6 --lazy --iters 10 2>&1 | grep resunit | sed "s/^/t16=$t16 /" | tee -a $O/ru48.txt
    done
  done
done
echo done
