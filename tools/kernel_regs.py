"""Register / LDS / spill summary of the gfx950 kernels in a built object (its .hip_fatbin), from the code
object's metadata notes.  usage: python tools/kernel_regs.py audiotokenization_amd/_build/resunit_x6.o [substring]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(path):
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "dev.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", path, os.path.join(td, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                              text=True).stdout


def kernels(text):
    cur = {}
    for line in text.splitlines():
        m = re.match(r"(\s+)(- )?\.(\w+):\s*(.*)$", line)
        if not m:
            continue
        ind, dash, k, v = m.groups()
        if dash and k == "agpr_count":  # first (sorted) key of a kernel's map
            if cur.get(".name"):
                yield cur
            cur = {}
        if "." + k not in cur:
            cur["." + k] = v.strip()
    if cur.get(".name"):
        yield cur


if __name__ == "__main__":
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for k in kernels(notes(sys.argv[1])):
        name = subprocess.run(["c++filt", k[".name"]], capture_output=True, text=True).stdout.strip()
        if pat in name:
            print(f"vgpr {k.get('.vgpr_count', '?'):>4} agpr {k.get('.agpr_count', '?'):>4} "
                  f"vspill {k.get('.vgpr_spill_count', '?'):>3} sspill {k.get('.sgpr_spill_count', '?'):>3} "
                  f"lds {k.get('.group_segment_fixed_size', '?'):>6}  {name}")
