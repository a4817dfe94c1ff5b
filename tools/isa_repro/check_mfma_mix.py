"""ISA lint for the resunit_rr hazard: an MFMA whose SrcC is EXACTLY the vDST of a recent MFMA of a
DIFFERENT opcode.  hipcc (ROCm 7.2, gfx950) treats an exact SrcC overlap as forwardable and inserts no wait state
for it (tools/isa_repro/mfma_chain.hip shows 0 between v_mfma_f32_16x16x32_f16 and a dependent
v_mfma_f32_16x16x16_f16), while resunit_rr observed intermittently wrong lanes with exactly that chain.  The
product kernels must not contain it: this scans every kernel's straight-line code (the previous 8 instructions).

usage: python tools/isa_repro/check_mfma_mix.py <obj.o|.so|.dis> [...]"""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import check_vmcnt as cv  # noqa: E402

_mfma = re.compile(r"^(v_mfma_\w+)\s+(\S+),\s*(\S+),\s*(\S+),\s*(\S+)")


def scan(dis):
    bad = []
    for name, base, body in cv.functions(dis):
        recent = []  # (index, opcode, vdst)
        for i, (addr, text, _) in enumerate(body):
            m = _mfma.match(text)
            if not m:
                continue
            op, vdst, srcc = m.group(1), m.group(2), m.group(5)
            for j, op1, vd1 in recent:
                if i - j <= 8 and vd1 == srcc and op1 != op:
                    bad.append(f"{name}+0x{addr - base:x}: {op} SrcC {srcc} = vDST of {op1} {i - j} instructions back")
            recent = [r for r in recent if r[2] != vdst] + [(i, op, vdst)]
    return bad


def main(argv):
    total = 0
    for p in argv:
        bad = scan(cv.disassemble(p))
        for b in bad:
            print("MIXED-CHAIN", b)
        total += len(bad)
        print(f"{os.path.basename(p)}: {len(bad)} mixed-opcode SrcC chains")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
