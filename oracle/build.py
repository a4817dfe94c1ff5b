"""Build the C oracle (oracle/vq_oracle.c -> oracle/_build/libvq_oracle.so) — test infrastructure.

The reference (hoyso48/AudioTokenization) is pure Python/PyTorch: it has no C/C++ sources, so there
is no oracle/_ref build; the Python oracle (bigcodec_oracle.py) runs on the reference's own torch
CPU ops and is pinned against fixtures the reference produced (tools/make_golden.py)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libvq_oracle.so")


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "vq_oracle.c")
    os.makedirs(OUT_DIR, exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(src):
        return LIB
    cmd = ["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared", src, "-o", LIB, "-lm"]
    subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
