"""ISA audits of the built HIP objects (tools/check_vmcnt.py, tools/isa_repro/check_mfma_mix.py):

  * every hand-counted `s_waitcnt vmcnt(N)` that follows an LDS-DMA weight copy must find that copy retired, i.e.
    the compiler must have issued every input load the count assumes AFTER the copy; in the
    pre-split projection GEMM, whose counted wait leaves the next chunk's two B copies in flight on purpose, the
    two youngest vm ops must be those copies and every older copy must retire;
  * no MFMA may read as SrcC the vDST of a recent MFMA of ANOTHER opcode: hipcc (ROCm 7.2) puts no wait state
    between them (it treats an exact SrcC overlap as forwarded), and on the MI355X that chain needs 4-5 wait states
    (tools/isa_repro/run_chain_probe.py: 16x16x16 -> 16x16x32 wrong on ~99 % of waves below 5 states, 16x16x32 ->
    16x16x16 on a few waves in 16 384 below 4) -- the cause of resunit_rr's "intermittently wrong lanes" (ADVICE r02)."""
import concurrent.futures as cf
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "audiotokenization_amd", "_build")
OBJECTS = ["conv1d_x6_p1.o", "conv1d_x6_p2.o", "conv1d_x6_p3.o", "resunit_x6.o", "pw_presplit.o"]
MFMA_OBJECTS = ["conv1d.o", "conv1d_x6_p1.o", "conv1d_x6_p2.o", "conv1d_x6_p3.o", "resunit_x6.o", "resunit_rr.o",
                "lstm.o", "lstm_seq.o", "vq.o", "elementwise.o", "resample.o", "probe.o", "pw_presplit.o"]
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "tools", "isa_repro"))


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


def _mix(obj):
    import check_mfma_mix as cm
    import check_vmcnt as cv

    return obj, cm.scan(cv.disassemble(os.path.join(BUILD, obj)))


def test_no_mixed_opcode_mfma_accumulator_chains():
    import check_vmcnt as cv

    missing = [o for o in MFMA_OBJECTS if not os.path.exists(os.path.join(BUILD, o))]
    if missing or not os.path.exists(os.path.join(cv.LLVM, "llvm-objdump")):
        pytest.skip(f"built objects / ROCm llvm tools not present ({missing})")
    with cf.ProcessPoolExecutor(max_workers=4) as ex:
        results = list(ex.map(_mix, MFMA_OBJECTS))
    bad = [b for _, found in results for b in found]
    assert not bad, "\n".join(bad[:10])


def _fake_kernel(name, ops):
    lines = [f"0000000000001000 <{name}>:"]
    for i, op in enumerate(ops):
        lines.append(f"\t{op} // {0x1000 + 8 * i:012X}: ")
    lines.append(f"\ts_endpgm // {0x1000 + 8 * len(ops):012X}: ")
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("ops,bad", [
    # A copy, then the two B copies, counted wait: the A copy retires, B(c + 2) stays in flight
    (["global_load_lds_dwordx4 v[0:1], off", "global_load_lds_dwordx4 v[2:3], off",
      "global_load_lds_dwordx4 v[4:5], off", "s_waitcnt vmcnt(2)"], False),
    # a load between the B copies: the youngest two vm ops are not both copies
    (["global_load_lds_dwordx4 v[0:1], off", "global_load_lds_dwordx4 v[2:3], off",
      "global_load_dword v6, v[8:9], off", "global_load_lds_dwordx4 v[4:5], off", "s_waitcnt vmcnt(2)"], True),
    # the count too large: the A copy is among the 3 youngest
    (["global_load_lds_dwordx4 v[0:1], off", "global_load_lds_dwordx4 v[2:3], off",
      "global_load_lds_dwordx4 v[4:5], off", "s_waitcnt vmcnt(3)"], True),
])
def test_in_flight_copy_rule_on_synthetic_code(ops, bad):
    """check_vmcnt's expected-in-flight rule (pw_presplit_kernel: two copies) on hand-made instruction streams."""
    import check_vmcnt as cv

    (name, base, body), = list(cv.functions(_fake_kernel("pw_presplit_kernel", ops)))
    _, hz = cv.audit(name, base, body)
    assert bool(hz) == bad, hz
    # the same stream plus an input load in a kernel with no expected in-flight copies: a copy among the counted
    # ops is a hazard
    ops0 = ops[:-1] + ["global_load_dword v6, v[8:9], off", ops[-1]]
    (name, base, body), = list(cv.functions(_fake_kernel("conv1d_x6_kernel", ops0)))
    assert cv.audit(name, base, body)[1]
