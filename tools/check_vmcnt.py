"""ISA audit of hand-counted `s_waitcnt vmcnt(N)` waits after LDS-DMA copies.

The conv / ResidualUnit kernels issue the next K-step's weight copy with `global_load_lds` (LDS-DMA) and then the
next chunk's input loads, and wait with `s_waitcnt vmcnt(2*CI)` so that only the younger input loads may stay in
flight.  That count is right only if no LDS-DMA copy is among the N youngest outstanding vector-memory operations
at the wait, i.e. if the compiler kept every later buffer load behind the copy.  vmcnt retires in issue order, so
after `s_waitcnt vmcnt(N)` an operation is still pending only if fewer than N operations were issued after it.

This script extracts the gfx950 code object from a built object / shared library (or reads a disassembly),
builds each kernel's control-flow graph and propagates, per instruction, the set of possible "number of vector
memory operations issued after the youngest LDS-DMA copy still outstanding" (None = none outstanding).  A wait
vmcnt(N) with N > 0 is a HAZARD if on some path an LDS-DMA copy is among its N youngest operations.

usage: python tools/check_vmcnt.py <file.o|.so|.dis> [...]   (exit status 1 if any hazard is found)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
CAP = 64

_vm_dma = re.compile(r"^\s*(global_load_lds|buffer_load_\w+.*\blds\b)")
_vm_op = re.compile(r"^\s*(global_|buffer_|flat_|scratch_)(load|store|atomic)")
_wait = re.compile(r"^\s*s_waitcnt\b(.*?)(//|$)")
_vmcnt = re.compile(r"vmcnt\((\d+)\)")
_fn = re.compile(r"^([0-9a-f]+) <(\S+)>:$")
_ins = re.compile(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):")
_tgt = re.compile(r"<(\S+)\+0x([0-9a-f]+)>\s*$")
_PW = re.compile(r"conv1d_x6_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi\d+ELb1E")  # PW = true instantiations


def disassemble(path: str) -> str:
    if path.endswith(".dis") or path.endswith(".s"):
        with open(path) as fh:
            return fh.read()
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", path, os.path.join(td, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                              capture_output=True, text=True).stdout


def functions(dis: str):
    cur, base, body = None, 0, []
    for line in dis.splitlines():
        m = _fn.match(line)
        if m:
            if cur:
                yield cur, base, body
            cur, base, body = m.group(2), int(m.group(1), 16), []
            continue
        m = _ins.match(line)
        if cur and m:
            body.append((int(m.group(2), 16), m.group(1), line))
    if cur:
        yield cur, base, body


# Kernels whose counted waits leave LDS-DMA copies in flight ON PURPOSE, with how many: the pre-split
# projection GEMM (csrc/pw_presplit.hip) issues, per chunk, A(c + 1) then exactly two B(c + 2) pieces per wave and
# waits vmcnt(2): the two youngest vm ops must be those copies (a load or a reordered copy there fails), and
# every older copy must retire.  (A reordering of A(c + 1) behind B(c + 2) keeps two copies youngest and is not
# visible here; the source pins that order with dma_issue_order().)
IN_FLIGHT_COPIES = [(re.compile(r"pw_presplit_kernel"), 2)]


def expected_in_flight(name: str) -> int:
    for pat, n in IN_FLIGHT_COPIES:
        if pat.search(name):
            return n
    return 0


def audit(name: str, base: int, body):
    """Returns (number of counted waits, [hazard descriptions]) for one kernel."""
    if not any(_vm_dma.match(t) for _, t, _ in body):
        return 0, []
    E = expected_in_flight(name)
    idx = {addr: i for i, (addr, _, _) in enumerate(body)}
    succ = []
    for i, (addr, text, line) in enumerate(body):
        op = text.split()[0]
        s = []
        m = _tgt.search(line)
        if op.startswith("s_cbranch") or op == "s_branch":
            if m and m.group(1) == name:
                t = base + int(m.group(2), 16)
                if t in idx:
                    s.append(idx[t])
        if op not in ("s_branch", "s_endpgm", "s_setpc_b64") and i + 1 < len(body):
            s.append(i + 1)
        succ.append(s)
    # state (ds, k): ds = for the E + 1 youngest LDS-DMA copies still pending, youngest first, the vm ops issued
    # after each (empty: none pending; E = 0 keeps one distance, "d"); k = vm loads (not copies) issued since the
    # last vmcnt wait or barrier (capped): loads placed IN FRONT of a copy within its K-step
    states = [set() for _ in body]
    states[0].add(((), 0))
    work = [0]
    hazards, counted, hoisted = [], set(), set()
    while work:
        i = work.pop()
        addr, text, _ = body[i]
        outs = set()
        for ds, k in states[i]:
            if _vm_dma.match(text):
                if k > 0:
                    hoisted.add((addr, text, k))
                ds = ((0,) + tuple(min(d + 1, CAP) for d in ds))[:E + 1]
            elif _vm_op.match(text):
                ds = tuple(min(d + 1, CAP) for d in ds)
                k = min(k + 1, CAP) if "load" in text.split()[0] else k
            elif text.startswith("s_barrier"):
                k = 0
            else:
                w = _wait.match(text)
                if w:
                    m = _vmcnt.search(w.group(1))
                    if m:
                        n = int(m.group(1))
                        if n > 0:
                            counted.add(i)
                            if E == 0:
                                if ds and ds[0] < n:
                                    hazards.append((addr, text, ds[0]))
                            else:
                                # the E youngest vm ops must be copies (the E youngest copies at distances 0..E-1)
                                # and the copy before them must retire at this count
                                if len(ds) >= E and tuple(ds[:E]) != tuple(range(E)):
                                    hazards.append((addr, text, -1))
                                if len(ds) > E and ds[E] < n:
                                    hazards.append((addr, text, ds[E]))
                        ds = tuple(d for d in ds if d < n)
                        k = 0
            outs.add((ds, k))
        for j in succ[i]:
            if not outs <= states[j]:
                states[j] |= outs
                work.append(j)
    # A pending copy with NO younger op (d = 0) at a counted wait is the path that issued a copy but skipped the
    # input loads: the kernels guard the count with the same condition as those loads (the other path waits
    # vmcnt(0)), so it is infeasible -- provided no load was placed in front of any copy (hoisted is empty).
    # Any d > 0 below the count, or any hoisted load, is a real ordering hazard.
    real = sorted({h for h in hazards if h[2] > 0})
    out = [f"{name}+0x{a - base:x}: {t}: an LDS-DMA copy with only {d} younger vm ops is still pending"
           for a, t, d in real]
    out += [f"{name}+0x{a - base:x}: {t}: the {E} youngest vm ops are not all LDS-DMA copies"
            for a, t, d in sorted({h for h in hazards if h[2] == -1})]
    # The pointwise conv path (conv1d_x6_kernel<..., PW = true, ...>) issues chunk 1's input loads in the
    # prologue, ahead of chunk 1's weight copy, by design: they are OLDER than the copy and retire before it
    # at the counted wait, so loads in front of a copy are expected there (and only there).
    if not _PW.search(name):
        out += [f"{name}+0x{a - base:x}: {t}: {k} vm loads issued in front of this LDS-DMA copy since the last wait"
                f" / barrier" for a, t, k in sorted(hoisted)]
    return len(counted), out


def main(argv):
    bad = 0
    for path in argv:
        dis = disassemble(path)
        nk = nw = 0
        for name, base, body in functions(dis):
            c, hz = audit(name, base, body)
            if c or hz:
                nk += 1
                nw += c
            for h in hz:
                print("HAZARD", h)
                bad += 1
        print(f"{os.path.basename(path)}: {nk} kernels with LDS-DMA and counted waits, {nw} counted waits, "
              f"{bad} hazards so far")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
