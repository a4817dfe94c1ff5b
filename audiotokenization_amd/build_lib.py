"""Build libbigcodec_hip.so (gfx950) in-tree with hipcc, and libbigcodec_ops.so (the torch.ops.bigcodec.*
custom operators over its C ABI) with g++ against the installed PyTorch-ROCm headers.

The shared library is the product: every compute kernel of the BigCodec path lives in
audiotokenization_amd/csrc/*.hip and is exported through the C ABI in include/bigcodec.h;
csrc/torch_ops.cpp registers that ABI with the PyTorch dispatcher (TORCH_LIBRARY(bigcodec)).
Built objects stay in-tree (git-ignored) so they travel with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD = os.path.join(PKG_DIR, "_build")
LIB = os.path.join(PKG_DIR, "libbigcodec_hip.so")
OPS_LIB = os.path.join(PKG_DIR, "libbigcodec_ops.so")
OPS_SRC = "torch_ops.cpp"
ARCH = os.environ.get("BIGCODEC_ARCH", "gfx950")

SOURCES = ["conv1d.hip", "conv1d_x6.hip", "conv1d_x6_p1.hip", "conv1d_x6_p2.hip", "conv1d_x6_p3.hip", "conv1d_x6ra.hip", "resunit_x6.hip", "resunit_w16.hip", "resunit_rr.hip", "elementwise.hip", "lstm.hip", "lstm_seq.hip", "pw_presplit.hip",
           "vq.hip", "resample.hip", "probe.hip", "abi.hip", "flac.cpp"]
HEADERS = ["bc_common.h", "bc_internal.h", "conv_epilogue.h", "x6_common.h", "conv1d_x6_kernel.h"]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
          "-Wall", "-Wno-unused-function", "-I", os.path.join(REPO, "include")]
if os.environ.get("BIGCODEC_ABLATION") == "1":  # tools/*_ablation.sh only: compiles the work-skipping switches in
    CFLAGS.append("-DBC_ABLATION")
if os.environ.get("BIGCODEC_NO_XCD_REMAP") == "1":  # experiment builds only: workgroups in the dispatcher's order
    CFLAGS.append("-DBC_NO_XCD_REMAP")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the BigCodec HIP library cannot be built")


DEBUG_DIR = os.path.join(PKG_DIR, "_debug")


def _paths(debug: bool):
    """(build dir, library, flags) of the product build or of the bounds-checked debug build (-DBC_DEBUG, in
    _debug/ next to its own copy of the torch ops library, loaded by the package when BIGCODEC_DEBUG=1)."""
    if debug:
        return os.path.join(DEBUG_DIR, "_build"), os.path.join(DEBUG_DIR, "libbigcodec_hip.so"), CFLAGS + ["-DBC_DEBUG"]
    return BUILD, LIB, CFLAGS


DIGEST_MARK = b"BC_BUILD_DIGEST="


def lib_digest(lib_path: str) -> str | None:
    """The source digest compiled INTO a built library (bc_build_digest; the marker string in its .rodata), read
    from the file without loading it; None for a missing file or a library without the marker."""
    try:
        with open(lib_path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(DIGEST_MARK)
    if i < 0:
        return None
    d = data[i + len(DIGEST_MARK):i + len(DIGEST_MARK) + 64]
    return d.decode() if len(d) == 64 and all(c in b"0123456789abcdef" for c in d) else None


def _digest(flags=None) -> str:
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(REPO, "include", "bigcodec.h"), "rb") as fh:
        h.update(fh.read())
    h.update(" ".join(flags or CFLAGS).replace(REPO, "<repo>").encode())  # (the tree moves: gpurun, the driver)
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False, debug: bool = False) -> str:
    """Compile (if sources changed) and return the path of libbigcodec_hip.so (debug: the bounds-checked build)."""
    build_dir, lib_path, flags = _paths(debug)
    os.makedirs(build_dir, exist_ok=True)
    dig = _digest(flags)
    # the digest lives in the library itself (no side stamp file that a checkout could leave agreeing with the
    # sources while the git-ignored .so is another tree's: ADVICE r04)
    if not force and lib_digest(lib_path) == dig:
        return lib_path
    hipcc = _hipcc()

    common = hashlib.sha256()  # every header (any source may include any of them) + the flags
    for f in HEADERS:
        with open(os.path.join(CSRC, f), "rb") as fh:
            common.update(fh.read())
    with open(os.path.join(REPO, "include", "bigcodec.h"), "rb") as fh:
        common.update(fh.read())
    common.update(" ".join(flags).encode())

    def compile_one(src: str) -> str:
        obj = os.path.join(build_dir, os.path.splitext(src)[0] + ".o")
        h = common.copy()
        with open(os.path.join(CSRC, src), "rb") as fh:
            h.update(fh.read())
        ostamp = obj + ".stamp"
        if not force and os.path.exists(obj) and os.path.exists(ostamp):
            with open(ostamp) as fh:
                if fh.read().strip() == h.hexdigest():
                    return obj  # unchanged source and headers: keep the object
        cmd = [hipcc, *flags, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{res.stderr}")
        with open(ostamp, "w") as fh:
            fh.write(h.hexdigest())
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 8, 16)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    # bc_build_digest (include/bigcodec.h): the digest of exactly these sources and flags, compiled in
    dsrc, dobj = os.path.join(build_dir, "digest.c"), os.path.join(build_dir, "digest.o")
    with open(dsrc, "w") as fh:
        fh.write(f'static const char bc_digest_str[] = "{DIGEST_MARK.decode()}{dig}";\n'
                 f'const char* bc_build_digest(void) {{ return bc_digest_str + {len(DIGEST_MARK)}; }}\n')
    res = subprocess.run([os.environ.get("CC", "gcc"), "-O2", "-fPIC", "-c", dsrc, "-o", dobj], capture_output=True,
                         text=True)
    if res.returncode != 0:
        raise RuntimeError(f"digest object failed:\n{res.stderr}")
    objs.append(dobj)
    tmp = lib_path + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,-soname,libbigcodec_hip.so", *objs, "-o", tmp]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"link failed:\n{res.stderr}")
    os.replace(tmp, lib_path)
    return lib_path


def _ops_flags(debug: bool = False):
    import torch
    import torch.utils.cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths(device_type="cuda")] + ["-I", os.path.join(REPO, "include")]
    libs = [f"-L{p}" for p in ce.library_paths(device_type="cuda")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return (["-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
             f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=bigcodec_ops"] + inc,
            libs + ["-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", f"-L{DEBUG_DIR if debug else PKG_DIR}", "-lbigcodec_hip",
                    "-Wl,-rpath,$ORIGIN"], torch.__version__)


def build_ops(force: bool = False, verbose: bool = False, debug: bool = False) -> str:
    """Compile csrc/torch_ops.cpp (if it, the header or torch changed) into libbigcodec_ops.so (debug: the copy in
    _debug/ that links the bounds-checked libbigcodec_hip.so next to it)."""
    build(verbose=verbose, debug=debug)
    cflags, ldflags, tv = _ops_flags(debug)
    h = hashlib.sha256()
    for f in (os.path.join(CSRC, OPS_SRC), os.path.join(REPO, "include", "bigcodec.h")):
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update((" ".join(cflags + ldflags) + tv).encode())
    dig = h.hexdigest()
    ops_lib = os.path.join(DEBUG_DIR, "libbigcodec_ops.so") if debug else OPS_LIB
    stamp = os.path.join(_paths(debug)[0], "ops_stamp")
    if not force and os.path.exists(ops_lib) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == dig:
                return ops_lib
    cxx = os.environ.get("CXX", "g++")
    tmp = ops_lib + ".tmp"
    cmd = [cxx, *cflags, os.path.join(CSRC, OPS_SRC), "-o", tmp, *ldflags]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"{cxx} failed for {OPS_SRC}:\n{res.stderr}")
    os.replace(tmp, ops_lib)
    with open(stamp, "w") as fh:
        fh.write(dig)
    return ops_lib


if __name__ == "__main__":  # python audiotokenization_amd/build_lib.py [--force] [--debug]
    dbg = "--debug" in sys.argv
    print(build(force="--force" in sys.argv, verbose=True, debug=dbg))
    print(build_ops(force="--force" in sys.argv, verbose=True, debug=dbg))
