"""The bounds-checked debug build (include/bigcodec.h bc_debug_status) on the MI355X.

audiotokenization_amd/_debug/libbigcodec_hip.so (build_lib.build(debug=True), prebuilt on the CPU like the product
library) is loaded by a child process with BIGCODEC_DEBUG=1:
  * bc_debug_selftest(n) makes n lanes fail a check on purpose: bc_debug_status reports exactly n failures and the
    check's line, and clears them;
  * the encode -> VQ -> decode of a small batch in h3 and x6, plus the conv / ResidualUnit / ResLSTM shapes of the
    encoder, run with every computed global access checked: 0 failures, and the outputs equal the product build's.
Skipped when the debug library is absent or older than the sources (it is a developer tool, not the product).
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

CHILD = r"""
import json, sys, torch
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r})
from audiotokenization_amd import _lib as L
from helpers import build_models
from audiotokenization_amd import synth
lib = L.load()
assert L.lib_path().endswith("_debug/libbigcodec_hip.so"), L.lib_path()
out = {{}}
L.call("bc_debug_selftest", 300, torch.cuda.current_stream().cuda_stream)
out["selftest"] = L.debug_status()
out["after"] = L.debug_status()
dev = torch.device("cuda", 0)
enc, dec, *_ = build_models("base", device=dev)
x = torch.from_numpy(synth.synth_clips(2, 12000, clip0=5)).unsqueeze(1).to(dev)
for prec in ("h3", "x6"):
    L.set_precision(prec)
    with torch.no_grad():
        post, codes, _ = dec(enc(x), vq=True)
        wav = dec(post, vq=False)
    out[prec] = L.debug_status()
    torch.save({{"codes": codes.cpu(), "wav": wav.cpu()}}, {dump!r} + prec + ".pt")
print("DEBUG_RESULT " + json.dumps(out))
"""


def test_debug_build_checks_and_selftest(tmp_path):
    sys.path.insert(0, REPO)
    from audiotokenization_amd import build_lib

    dlib = os.path.join(build_lib.DEBUG_DIR, "libbigcodec_hip.so")
    if not os.path.exists(dlib):
        pytest.skip("debug library not built (python audiotokenization_amd/build_lib.py --debug)")
    # the digest compiled into the library itself (bc_build_digest), not a side file
    if build_lib.lib_digest(dlib) != build_lib._digest(build_lib._paths(True)[2]):
        pytest.skip("debug library older than the sources")
    dump = str(tmp_path / "dbg_")
    code = CHILD.format(repo=REPO, tests=os.path.join(REPO, "tests"), dump=dump)
    env = dict(os.environ, BIGCODEC_DEBUG="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("DEBUG_RESULT ")][-1]
    res = json.loads(line[len("DEBUG_RESULT "):])
    print(res)
    assert res["selftest"][0] == 300 and res["selftest"][1] > 0, res
    assert res["after"] == [0, 0], res
    assert res["h3"] == [0, 0] and res["x6"] == [0, 0], res
    # the checked build computes what the product build computes
    import torch

    from audiotokenization_amd import _lib as L
    from audiotokenization_amd import synth
    from helpers import build_models

    dev = torch.device("cuda", 0)
    enc, dec, *_ = build_models("base", device=dev)
    x = torch.from_numpy(synth.synth_clips(2, 12000, clip0=5)).unsqueeze(1).to(dev)
    old = L.precision_mode()
    try:
        for prec in ("h3", "x6"):
            L.set_precision(prec)
            with torch.no_grad():
                post, codes, _ = dec(enc(x), vq=True)
                wav = dec(post, vq=False)
            d = torch.load(dump + prec + ".pt", weights_only=True)
            assert torch.equal(d["codes"], codes.cpu()), prec
            assert torch.equal(d["wav"], wav.cpu()), prec
    finally:
        L._mode = old
