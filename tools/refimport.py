"""Import the reference BigCodec hot-path modules from /root/reference (fixture generation only).

This helper exists only in the development container: /root/reference is never present on the GPU
box and nothing under tests/ that runs there imports this file.  The reference package
`vq/__init__.py` pulls in the vendored lucidrains library, which needs `einx` (absent here), so we
register a bare `vq` package (skipping its __init__) and a stub for the lucidrains sub-package whose
FSQ is the real class (its file has no einx dependency; load_fsq); VectorQuantize stays a stub (unused
by BigCodec).
"""
import importlib
import os
import sys
import types

REF_ROOT = os.environ.get("BIGCODEC_REF_ROOT", "/root/reference/BigCodec_SSL")


def available() -> bool:
    return os.path.isfile(os.path.join(REF_ROOT, "vq", "codec_encoder.py"))


def load_fsq():
    """The reference's vendored FSQ module (vq/vector_quantize_pytorch_lucidrains/
    finite_scalar_quantization.py), loaded as a standalone file: it needs torch and einops only, not
    the package __init__ (which needs einx)."""
    import importlib.util

    name = "vq_lucid_finite_scalar_quantization"
    if name in sys.modules:
        return sys.modules[name]
    path = os.path.join(REF_ROOT, "vq", "vector_quantize_pytorch_lucidrains", "finite_scalar_quantization.py")
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load():
    """Return (codec_encoder, codec_decoder, residual_vq, fvq, module, activations, alias_free) modules."""
    if not available():
        raise RuntimeError(f"reference not found at {REF_ROOT}")
    if "vq" not in sys.modules or not getattr(sys.modules["vq"], "_graft_stub", False):
        pkg = types.ModuleType("vq")
        pkg.__path__ = [os.path.join(REF_ROOT, "vq")]
        pkg._graft_stub = True
        sys.modules["vq"] = pkg
        lucid = types.ModuleType("vq.vector_quantize_pytorch_lucidrains")
        lucid.VectorQuantize = None
        lucid.FSQ = load_fsq().FSQ  # its file imports only torch / einops: loaded on its own
        sys.modules["vq.vector_quantize_pytorch_lucidrains"] = lucid
    enc = importlib.import_module("vq.codec_encoder")
    dec = importlib.import_module("vq.codec_decoder")
    rvq = importlib.import_module("vq.residual_vq")
    fvq = importlib.import_module("vq.factorized_vector_quantize")
    mod = importlib.import_module("vq.module")
    act = importlib.import_module("vq.activations")
    af = importlib.import_module("vq.alias_free_torch")
    return types.SimpleNamespace(encoder=enc, decoder=dec, rvq=rvq, fvq=fvq, module=mod,
                                 activations=act, alias_free=af)
