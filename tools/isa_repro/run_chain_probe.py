"""GPU check of the mixed MFMA chain (tools/isa_repro/mfma_chain.hip): the 16x16x32 -> dependent 16x16x16 chain as
hipcc emits it (no wait states) vs the same chain with 16 wait states between.  Equal bits on every wave mean the
hardware forwards the exact-overlap SrcC across the two opcodes; a difference means the wait states are required
and the compiler omits them.

usage: python tools/isa_repro/run_chain_probe.py [--build]   (--build compiles the .so here, on the CPU side)"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmfma_chain.so")


def build():
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-shared", "-fPIC",
                    os.path.join(HERE, "mfma_chain.hip"), "-o", SO], check=True)


def main():
    if "--build" in sys.argv:
        build()
        print("built", SO)
        return 0
    import torch

    lib = ctypes.CDLL(SO)
    waves = 16384
    g = torch.Generator().manual_seed(7)
    dev = torch.device("cuda", 0)
    a = torch.randn(waves * 64, 8, generator=g).half().to(dev)
    b = torch.randn(waves * 64, 8, generator=g).half().to(dev)
    c = torch.randn(waves * 64, 4, generator=g).half().to(dev)
    d = torch.randn(waves * 64, 4, generator=g).half().to(dev)
    names = {0: "16x16x32 -> 16x16x16", 1: "16x16x16 -> 16x16x32", 2: "16x16x32 -> 16x16x32"}
    bad_any = 0
    for order in (0, 1, 2):
        ref = torch.empty(waves * 64, 4, device=dev)
        assert lib.mfma_chain_probe(*(ctypes.c_void_p(t.data_ptr()) for t in (a, b, c, d, ref)), waves, order, 16) == 0
        for gap in (0, 1, 2, 3, 4, 5, 6, 8):
            worst = 0
            for rep in range(5):
                o = torch.empty_like(ref)
                assert lib.mfma_chain_probe(*(ctypes.c_void_p(t.data_ptr()) for t in (a, b, c, d, o)), waves, order,
                                            gap) == 0
                torch.cuda.synchronize()
                worst = max(worst, int((o != ref).any(dim=1).view(waves, 64).any(dim=1).sum()))
            bad_any += worst
            print(f"{names[order]}, {gap} wait states between: {worst} / {waves} waves differ from the 16-state chain",
                  flush=True)
    print(f"chain probe: {'wait states REQUIRED where rows above differ' if bad_any else 'no difference at any gap'}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
