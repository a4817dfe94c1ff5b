import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "reference: needs /root/reference (development container only)")


# GPU modules run from the kernel level up (a kernel regression is reported by its own test before any
# whole-model test trips over it), the full-size config runs last (they take the longest).  Stable: the
# order within a module is unchanged; modules not listed keep their place before the listed ones.
_GPU_ORDER = ["test_gpu_kernels", "test_gpu_ops", "test_gpu_fsq", "test_gpu_model", "test_gpu_tokens",
              "test_gpu_streaming", "test_gpu_extract", "test_extract_cli", "test_gpu_full_size",
              "test_gpu_configs"]


def pytest_collection_modifyitems(config, items):
    import torch

    has_gpu = torch.cuda.is_available()
    for item in items:
        if "gpu" in item.keywords and not has_gpu:
            item.add_marker(pytest.mark.skip(reason="no HIP device"))

    def key(item):
        mod = item.module.__name__.rsplit(".", 1)[-1] if item.module else ""
        return _GPU_ORDER.index(mod) + 1 if mod in _GPU_ORDER else 0
    items.sort(key=key)


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    out = {k: d[k] for k in d.files}
    if "meta" in out:
        out["meta"] = json.loads(str(out["meta"]))
    return out


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(params=["fp32", "x6", "h3"])
def prec(request):
    """Run a test under every fp32-class conv GEMM precision: native fp32 MFMA, the 3xbf16 split MFMA
    ("x6") and the 2xfp16 block-scaled split MFMA ("h3"), csrc/conv1d_x6.hip."""
    from audiotokenization_amd import _lib

    old = _lib.precision_mode()
    _lib.set_precision(request.param)
    yield request.param
    _lib._mode = old


@pytest.fixture(scope="session")
def dev():
    import torch

    from audiotokenization_amd import _lib

    _lib.load()  # the HIP library must load: no fallback
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _debug_build_bounds(request):
    """Under the bounds-checked debug build (BIGCODEC_DEBUG=1: `BIGCODEC_DEBUG=1 pytest -m gpu` runs every GPU test on
    it), a GPU test also fails when any kernel it launched counted a failed index check (include/bigcodec.h
    bc_debug_status); the product build compiles no checks and this is a no-op."""
    yield
    if os.environ.get("BIGCODEC_DEBUG") != "1" or "gpu" not in request.keywords:
        return
    import torch

    if not torch.cuda.is_available():
        return
    from audiotokenization_amd import _lib

    st = _lib.debug_status()
    assert st is None or st[0] == 0, f"debug build: {st[0]} failed index checks, first at source line {st[1]}"
