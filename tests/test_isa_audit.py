"""ISA audit of the built HIP objects: every hand-counted `s_waitcnt vmcnt(N)` that follows
an LDS-DMA weight copy must find that copy retired, i.e. the compiler must have issued every input load the count
assumes AFTER the copy (tools/check_vmcnt.py: CFG walk over the disassembled gfx950 code objects)."""
import concurrent.futures as cf
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "audiotokenization_amd", "_build")
OBJECTS = ["conv1d_x6_p1.o", "conv1d_x6_p2.o", "conv1d_x6_p3.o", "resunit_x6.o"]
sys.path.insert(0, os.path.join(REPO, "tools"))


def _audit(obj):
    import check_vmcnt as cv

    dis = cv.disassemble(os.path.join(BUILD, obj))
    kernels = waits = 0
    hazards = []
    for name, base, body in cv.functions(dis):
        c, hz = cv.audit(name, base, body)
        if c or hz:
            kernels += 1
            waits += c
        hazards += hz
    return obj, kernels, waits, hazards


def test_counted_vmcnt_waits_retire_the_lds_dma_copies():
    import check_vmcnt as cv

    missing = [o for o in OBJECTS if not os.path.exists(os.path.join(BUILD, o))]
    if missing or not os.path.exists(os.path.join(cv.LLVM, "llvm-objdump")):
        pytest.skip(f"built objects / ROCm llvm tools not present ({missing})")
    with cf.ProcessPoolExecutor(max_workers=4) as ex:
        results = list(ex.map(_audit, OBJECTS))
    total = 0
    for obj, kernels, waits, hazards in results:
        print(f"{obj}: {kernels} kernels with LDS-DMA copies, {waits} counted waits, {len(hazards)} hazards")
        assert kernels > 0 and waits > 0, f"{obj}: nothing audited (disassembly format changed?)"
        assert not hazards, "\n".join(hazards[:10])
        total += waits
    assert total > 500
