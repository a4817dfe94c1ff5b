"""The C-ABI library builds for gfx950, loads, and exports every symbol include/bigcodec.h declares;
host-side weight packing follows the documented layouts (no GPU needed)."""
import os
import re
import subprocess

import numpy as np
import pytest

from audiotokenization_amd import _lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(REPO, "include", "bigcodec.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(bc_[A-Za-z0-9_]+)\s*\(", txt)))


def test_library_loads_and_exports_all_declared_symbols():
    lib = L.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in L.EXPORTED, f"{s} missing from the ctypes signature table"
    assert set(L.EXPORTED) == set(syms)
    assert lib.bc_abi_version() == L.ABI_VERSION


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", L.lib_path()], capture_output=True, text=True)
    bundles = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                              f"--input={L.lib_path()}"], capture_output=True, text=True)
    assert "gfx950" in (out.stdout + bundles.stdout + open(L.lib_path(), "rb").read().decode("latin1"))


@pytest.mark.parametrize("Cout,Cin,K", [(48, 1, 7), (48, 48, 7), (96, 48, 4), (1536, 768, 10), (1, 32, 7), (6144, 1536, 1)])
def test_conv_pack_layout(Cout, Cin, K):
    lib = L.load()
    cfg = lib.bc_conv1d_select_cfg(Cout, Cin, K, 1, 1, 0)
    mt, wm, nt, wn, bkc = L.CONV_CFGS[cfg]
    n = lib.bc_conv1d_packed_floats(Cout, Cin, K, cfg)
    bm = 16 * mt * wm
    ntm = -(-Cout // bm)
    nch = -(-Cin // bkc)
    nks = bkc * K // 4
    assert n == ntm * wm * nch * nks * 64 * 4
    rng = np.random.default_rng(0)
    w = rng.standard_normal((Cout, Cin, K)).astype(np.float32)
    out = np.empty(n, np.float32)
    assert lib.bc_conv1d_pack(w.ctypes.data, out.ctypes.data, Cout, Cin, K, cfg) == 0
    P = out.reshape(ntm * wm, nch, nks, 64, 4)
    for _ in range(200):  # random element checks against the documented layout
        mg, c, ks, lane, i = (rng.integers(s) for s in P.shape)
        row = mg * 16 * mt + i * 16 + (lane & 15)
        kidx = ks * 4 + (lane >> 4)
        tap, ci = kidx // bkc, c * bkc + kidx % bkc
        want = w[row, ci, tap] if (i < mt and row < Cout and ci < Cin) else 0.0
        assert P[mg, c, ks, lane, i] == want
    # every weight appears exactly once
    assert np.isclose(P.sum(dtype=np.float64), w.sum(dtype=np.float64), rtol=1e-6, atol=1e-3)


def _bf16_to_f64(h):
    return (h.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


@pytest.mark.parametrize("Cout,Cin,K", [(48, 48, 7), (96, 48, 4), (1536, 768, 10), (6144, 1536, 1), (20, 36, 5)])
def test_x6_pack_layout_and_exact_split(Cout, Cin, K):
    """x6 mode packs each weight as three bf16 planes w = h0 + h1 + h2 (exact), in the
    [mg][chunk][tap][plane][q][lane][8] order conv1d_x6.hip documents."""
    lib = L.load()
    cfg = lib.bc_conv1d_select_cfg(Cout, Cin, K, 1, 1, 1)
    assert cfg in L.X6_CFGS
    mt, nt, wm, wn = L.X6_CFGS[cfg]
    bm, qa = 16 * mt * wm, mt * wm
    ntm, nch = -(-Cout // bm), -(-Cin // 32)
    n = lib.bc_conv1d_packed_floats(Cout, Cin, K, cfg)
    assert n * 4 == ntm * nch * K * 3 * qa * 1024
    rng = np.random.default_rng(1)
    w = (rng.standard_normal((Cout, Cin, K)) * np.exp(rng.standard_normal((Cout, 1, 1)) * 3)).astype(np.float32)
    out = np.empty(n, np.float32)
    assert lib.bc_conv1d_pack(w.ctypes.data, out.ctypes.data, Cout, Cin, K, cfg) == 0
    P = out.view(np.uint16).reshape(ntm, nch, K, 3, qa, 64, 8)
    planes = _bf16_to_f64(P)
    total = planes.sum(axis=3)  # (ntm, nch, K, qa, 64, 8)
    for _ in range(300):
        mg, c, tap, q, lane, j = (rng.integers(s) for s in total.shape)
        row = mg * bm + q * 16 + (lane & 15)
        ci = c * 32 + 8 * (lane >> 4) + j
        want = float(w[row, ci, tap]) if (row < Cout and ci < Cin) else 0.0
        assert total[mg, c, tap, q, lane, j] == want
        # each plane is the bf16 rounding of the remainder of the previous ones (|h1| <= ulp_bf16(h0)/2 ...)
        h0, h1 = planes[mg, c, tap, 0, q, lane, j], planes[mg, c, tap, 1, q, lane, j]
        assert abs(h1) <= abs(h0) * 2.0 ** -8
    assert np.array_equal(np.sort(total.reshape(-1)[total.reshape(-1) != 0]), np.sort(w.reshape(-1)[w.reshape(-1) != 0]).astype(np.float64))


def test_lstm_pack_layout():
    lib = L.load()
    H = 32
    w = np.arange(4 * H * H, dtype=np.float32).reshape(4 * H, H)
    for mode in (0, 1):  # H = 32: no persistent x6 kernel, both modes use the per-step layout
        out = np.empty(lib.bc_lstm_hh_packed_floats(H, mode), np.float32)
        assert lib.bc_lstm_pack_hh(w.ctypes.data, out.ctypes.data, H, mode) == 0
        P = out.reshape(H // 4, H // 4, 64)
        for ug, ks, lane in [(0, 0, 0), (3, 5, 17), (7, 7, 63)]:
            m = lane & 15
            assert P[ug, ks, lane] == w[(m >> 2) * H + ug * 4 + (m & 3), ks * 4 + (lane >> 4)]
        assert sorted(out.tolist()) == sorted(w.reshape(-1).tolist())


@pytest.mark.parametrize("H", [256, 512])
def test_lstm_seq_pack_layout(H):
    """mode 1: W_hh as three exact bf16 planes in the persistent kernel's register order
    [workgroup][wave][m-tile][k-step][plane][lane][8], m-tile rows unit-major (m = 4*unit + gate)."""
    lib = L.load()
    rng = np.random.default_rng(H)
    w = (rng.standard_normal((4 * H, H)) / np.sqrt(H)).astype(np.float32)
    n = lib.bc_lstm_hh_packed_floats(H, 1)
    assert n * 4 == 4 * H * H * 3 * 2
    out = np.empty(n, np.float32)
    assert lib.bc_lstm_pack_hh(w.ctypes.data, out.ctypes.data, H, 1) == 0
    KS, G = H // 128, H // 8
    planes = _bf16_to_f64(out.view(np.uint16).reshape(G, 4, 2, KS, 3, 64, 8))
    total = planes.sum(axis=4)
    for _ in range(300):
        g, wv, mt, ks, lane, j = (rng.integers(s) for s in total.shape)
        m = lane & 15
        row = (m & 3) * H + g * 8 + mt * 4 + (m >> 2)
        k = (wv * KS + ks) * 32 + 8 * (lane >> 4) + j
        assert total[g, wv, mt, ks, lane, j] == float(w[row, k])
    assert np.array_equal(np.sort(total.reshape(-1)), np.sort(w.reshape(-1).astype(np.float64)))


def test_bad_arguments_are_rejected_without_launching():
    lib = L.load()
    assert lib.bc_conv1d_select_cfg(0, 4, 7, 1, 1, 0) == -1
    assert lib.bc_conv1d_select_cfg(8, 4, 7, 1, 1, 4) == -1  # unknown precision mode
    assert lib.bc_conv1d_select_cfg(48, 48, 7, 1, 1, 2) >= 200  # bf16 products: one-plane tiles
    assert lib.bc_conv1d_select_cfg(8, 4, 7, 1, 1, 1) in L.CONV_CFGS  # x6 needs Cin >= 16: fp32 kernel
    assert lib.bc_conv1d_packed_floats(8, 8, 0, 0) == -1
    assert lib.bc_conv1d_fwd(None, None, None, None, None, None, None, None, 1, 8, 8, 8, 8, 3, 1, 1, 1, 0, 4,
                             None) == 1
    # dual output without an epilogue Snake, tanh together with a Snake: rejected
    assert lib.bc_conv1d_fwd(1, 1, None, None, None, None, 1, 1, 1, 8, 8, 8, 8, 3, 1, 1, 1, 0, 4, None) == 1
    assert lib.bc_lstm_hh_packed_floats(10, 0) == -1
    assert lib.bc_lstm_hh_packed_floats(512, 4) == -1
    assert lib.bc_vq_prepare_codebook(1, 1, 1, 8192, 16, None) == 3
    assert lib.bc_synth_clips(None, 1, 10, 0, None) == 1
    assert lib.bc_convT1d_phase_taps(10, 5) == 2 and lib.bc_convT1d_phase_taps(1, 1) == 1


def test_product_never_imports_oracle():
    pkg = os.path.join(REPO, "audiotokenization_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(root, f)).read()
                assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, flags=re.M), f


@pytest.mark.parametrize("Cout,Cin,K", [(48, 48, 7), (1536, 768, 10), (6144, 1536, 1), (20, 36, 5)])
def test_h3_pack_layout_and_scaled_split(Cout, Cin, K):
    """h3 mode (precision 3) packs each weight as two fp16 planes of w * S[row] (S = 2^(14 - e) with
    2^e <= max|w[row]| < 2^(e+1)), h0 = fp16(w S), h1 = fp16(w S - h0), in the x6 plane order, followed
    by 1 / S[row] for every packed row (conv1d_x6.hip, x6_common.h)."""
    lib = L.load()
    cfg = lib.bc_conv1d_select_cfg(Cout, Cin, K, 1, 1, 3)
    assert cfg % 1000 >= 300
    mt, nt, wm, wn = L.X6_CFGS[cfg % 100 + 100]
    bm, qa = 16 * mt * wm, mt * wm
    ntm, nch = -(-Cout // bm), -(-Cin // 32)
    n = lib.bc_conv1d_packed_floats(Cout, Cin, K, cfg)
    main = ntm * nch * K * 2 * qa * 1024
    assert n * 4 == main + ntm * bm * 4
    rng = np.random.default_rng(2)
    w = (rng.standard_normal((Cout, Cin, K)) * np.exp(rng.standard_normal((Cout, 1, 1)) * 6)).astype(np.float32)
    w[0] = 0.0  # an all-zero row keeps scale 1
    out = np.empty(n, np.float32)
    assert lib.bc_conv1d_pack(w.ctypes.data, out.ctypes.data, Cout, Cin, K, cfg) == 0
    P = out[: main // 4].view(np.float16).reshape(ntm, nch, K, 2, qa, 64, 8).astype(np.float64)
    inv = out[main // 4:].astype(np.float64)
    amax = np.abs(w).reshape(Cout, -1).max(axis=1).astype(np.float64)
    S = np.where(amax > 0, 2.0 ** (14 - np.floor(np.log2(np.where(amax > 0, amax, 1.0)))), 1.0)
    assert np.array_equal(inv[:Cout], 1.0 / S)
    assert (np.abs(w).reshape(Cout, -1).max(axis=1) * S < 2.0 ** 15).all()
    for _ in range(300):
        mg, c, tap, q, lane, j = (int(rng.integers(s)) for s in (ntm, nch, K, qa, 64, 8))
        row = mg * bm + q * 16 + (lane & 15)
        ci = c * 32 + 8 * (lane >> 4) + j
        h0, h1 = P[mg, c, tap, 0, q, lane, j], P[mg, c, tap, 1, q, lane, j]
        if row >= Cout or ci >= Cin:
            assert h0 == 0 and h1 == 0
            continue
        ws = float(w[row, ci, tap]) * S[row]
        assert h0 == float(np.float16(ws))
        assert abs(ws - h0 - h1) <= abs(ws) * 2.0 ** -22 + 2.0 ** -25


def test_torch_ops_registered_with_schemas_and_fakes():
    """torch.ops.bigcodec.* (csrc/torch_ops.cpp + ops.py): every op is registered, its schema names the
    ABI arguments, mutating ops mark their outputs (a!), and the fake kernels give the right shapes
    on meta tensors (no GPU needed)."""
    import torch

    from audiotokenization_amd import ops

    ns = ops.load()
    for name in ops.OPS:
        op = getattr(ns, name)
        schema = str(op.default._schema)
        assert schema.startswith(f"bigcodec::{name}("), schema
        if name.endswith("_"):
            assert "(a!)" in schema, schema
    m = lambda *s, dt=torch.float32: torch.empty(*s, device="meta", dtype=dt)  # noqa: E731
    w = m(10)
    assert [t.shape for t in ns.conv1d(m(2, 48, 1000), w, None, None, m(96), m(96), 96, 500, 4, 2, 1, 1, 0, 5, True)] \
        == [(2, 96, 500)] * 2
    assert ns.conv_transpose1d(m(2, 96, 10), [w, w], None, None, None, 48, 20, 4, 2, 1, 5, False)[0].shape == (2, 48, 20)
    assert [t.shape for t in ns.resunit(m(2, 48, 64), None, m(48), m(48), w, None, m(48), m(48), w, None, None, None,
                                        1, 3, 300, False)] == [(2, 48, 64)]
    assert ns.snake(m(2, 8, 5), m(8), m(8)).shape == (2, 8, 5)
    assert ns.tanh(m(3, 1, 7)).shape == (3, 1, 7)
    y, st, hT, cT = ns.reslstm(m(4, 512, 30), [w, w], [w, w], [w, w], None, None, 3, None, None, True)
    assert y.shape == (4, 512, 30) and st.dtype == torch.int32 and hT.shape == cT.shape == (2, 512, 4)
    idx, ze, post = ns.vq(m(2, 1024, 12), w, w, m(8192, 8), m(8192, 8), m(8192), w, w, True, True)
    assert idx.shape == (2, 12) and idx.dtype == torch.int64 and ze.shape == (2, 8, 12) and post.shape == (2, 1024, 12)
    assert ns.vq2emb(m(2, 12, 3, dt=torch.int64), 1, m(8192, 8), m(1024, 8), m(1024)).shape == (2, 12, 1024)
    assert ns.vq2emb_ct(m(2, 12, 3, dt=torch.int64), m(3, 8192, 8), m(3, 1024, 8), m(3, 1024)).shape == (2, 1024, 12)
    post, idx = ns.fsq(m(2, 512, 9), w, w, w, w, w)
    assert post.shape == (2, 512, 9) and idx.dtype == torch.int32
    tok = ns.fsq_codes(m(2, 9, dt=torch.int32), m(512, 4), m(512), [4, 4, 4, 8])
    assert tok.shape == (2, 512, 9) and tok.dtype == torch.float32
    win, nctx = ns.stream_window(m(2, 48, 100), m(2, 48, 18), m(48), m(48), 18)
    assert win.shape == (2, 48, 118) and nctx.shape == (2, 48, 18)
    assert ns.resample_sinc(m(3, 160), w, 240, 256, 2, 3, 16, 6).shape == (3, 256)


def test_torch_ops_library_links_the_abi_library():
    """libbigcodec_ops.so calls the C ABI of libbigcodec_hip.so (one instance, found next to it)."""
    from audiotokenization_amd import ops

    out = subprocess.run(["readelf", "-d", ops.OPS_PATH], capture_output=True, text=True).stdout
    assert "libbigcodec_hip.so" in out and "$ORIGIN" in out


def test_kernel_names_come_from_the_launchers():
    """bc_conv1d_kernel_name / bc_resunit_kernel_name (the roofline attribution) name the template the
    launcher instantiates for the selected cfg: the tile's template arguments and the plane count."""
    lib = L.load()
    for (Cout, Cin, K, s, d, mode) in [(384, 384, 7, 1, 9, 3), (768, 768, 1, 1, 1, 3), (768, 384, 10, 5, 1, 3),
                                       (192, 192, 7, 1, 3, 1), (96, 48, 4, 2, 1, 3), (48, 1, 7, 1, 1, 3)]:
        cfg = lib.bc_conv1d_select_cfg(Cout, Cin, K, s, d, mode)
        name = L.conv_kernel_name(cfg, K, s, d)
        base = cfg % 1000
        if 100 <= base < 400:
            mt, nt, wm, wn = L.X6_CFGS[base % 100 + 100]
            planes = {1: 3, 2: 1, 3: 2}[base // 100]
            assert name.startswith(f"conv1d_x6_kernel<{mt}, {nt}, {wm}, {wn}, {planes}, "), (cfg, name)
            # <..., planes, pointwise, taps per K-step, double-buffered B, 16-byte input staging>
            assert re.search(r", (true, 1, false|false, [124], (true|false)), (true|false)>$", name), name
        else:
            mt, wm, nt, wn, bkc = L.CONV_CFGS[cfg]
            assert name == f"conv1d_mfma_kernel<{mt}, {wm}, {nt}, {wn}, {bkc}>", name
    assert L.conv_kernel_name(lib.bc_conv1d_select_cfg(768, 768, 1, 1, 1, 3), 1).endswith("true, 1, false, true>")  # pointwise, B4
    # k7 C = 768: the 16-wave 192 x 256 tile, two taps per K-step, 16-byte input staging; the final k3 keeps the
    # double-buffered 256 x 256; the phase-decomposed stride-5 conv on the 16-wave tile stages single floats
    assert L.conv_kernel_name(lib.bc_conv1d_select_cfg(768, 768, 7, 1, 3, 3), 7, 1, 3) == \
        "conv1d_x6_kernel<6, 2, 2, 8, 2, false, 2, false, true>"
    assert L.conv_kernel_name(lib.bc_conv1d_select_cfg(1024, 1536, 3, 1, 1, 3), 3).endswith("false, 1, true, false>")
    assert L.conv_kernel_name(lib.bc_conv1d_select_cfg(768, 384, 10, 5, 1, 3), 10, 5, 1) == \
        "conv1d_x6_kernel<6, 2, 2, 8, 2, false, 2, false, false>"
    # x6 (the default): both stride-5 downsampling convs on the register-A tile (conv1d_x6ra.hip, round 5), the
    # stride-2 ones and the k7 / pointwise convs on the 16-wave tile, the final k3 on the 256 x 256 tile
    assert lib.bc_conv1d_select_cfg(768, 384, 10, 5, 1, 1) == 5120
    assert lib.bc_conv1d_select_cfg(1536, 768, 10, 5, 1, 1) == 5120
    assert L.conv_kernel_name(5120, 10, 5, 1) == "conv1d_x6ra_kernel<false>"
    assert lib.bc_conv1d_select_cfg(384, 192, 4, 2, 1, 1) == 2122
    assert L.conv_kernel_name(lib.bc_conv1d_select_cfg(384, 384, 7, 1, 9, 1), 7, 1, 9) == \
        "conv1d_x6_kernel<6, 2, 2, 8, 3, false, 1, false, true>"
    assert L.conv_kernel_name(lib.bc_conv1d_select_cfg(384, 384, 1, 1, 1, 1), 1) == \
        "conv1d_x6_kernel<6, 2, 2, 8, 3, true, 1, false, true>"
    assert lib.bc_conv1d_select_cfg(1024, 1536, 3, 1, 1, 1) == 121
    # bf16 on the 16-wave tile: four taps per K-step over the double B buffer
    assert L.conv_kernel_name(lib.bc_conv1d_select_cfg(384, 384, 7, 1, 3, 2), 7, 1, 3) == \
        "conv1d_x6_kernel<6, 2, 2, 8, 1, false, 4, true, true>"
    # C = 48 in h3: the streaming strip kernel (one per dilation); C = 96: the one-launch x6-family unit
    assert L.resunit_kernel_name(lib.bc_resunit_select_cfg(48, 1, 3), 48, 1) == "resunit_strip_kernel<1>"
    assert L.resunit_kernel_name(lib.bc_resunit_select_cfg(48, 9, 3), 48, 9) == "resunit_strip_kernel<9>"
    n96 = L.resunit_kernel_name(lib.bc_resunit_select_cfg(96, 3, 3), 96, 3)
    assert n96.startswith("resunit_x6_kernel<") and ", 2, " in n96, n96
    # bf16: the same unit with one bf16 plane (P = 1), at C = 48 too
    for C, d in ((48, 1), (96, 3)):
        nb = L.resunit_kernel_name(lib.bc_resunit_select_cfg(C, d, 2), C, d)
        assert nb.startswith("resunit_x6_kernel<") and re.search(r", 1, [124]>$", nb), nb
    # x6: the C = 48 unit at two taps per K-step, C = 96 at one, C = 192 the 16-wave unit; the x6 C = 32 / 16 tiles
    # launch one tap per K-step, and their names say so
    assert L.resunit_kernel_name(lib.bc_resunit_select_cfg(48, 3, 1), 48, 3) == "resunit_x6_kernel<3, 1, 1, 8, 3, 2>"
    assert L.resunit_kernel_name(lib.bc_resunit_select_cfg(96, 3, 1), 96, 3) == "resunit_x6_kernel<6, 1, 1, 8, 3, 1>"
    assert L.resunit_kernel_name(lib.bc_resunit_select_cfg(192, 3, 1), 192, 3).startswith("resunit_w16_kernel<3, ")
    assert L.resunit_kernel_name(lib.bc_resunit_select_cfg(192, 3, 2), 192, 3).startswith("resunit_w16_kernel<1, ")
    for C in (16, 32):
        nx = L.resunit_kernel_name(lib.bc_resunit_select_cfg(C, 3, 1), C, 3)
        assert re.search(r", 3, 1>$", nx), nx
    with pytest.raises(L.BigCodecLibraryError):
        L.conv_kernel_name(12345, 7)


def test_product_build_has_no_debug_checks():
    """bc_debug_status / bc_debug_selftest exist in every build; the product library answers 3 (unsupported):
    its index guards are compiled out (bc_common.h BC_DOK)."""
    import ctypes

    lib = L.load()
    out = (ctypes.c_uint * 2)(7, 7)
    assert lib.bc_debug_status(ctypes.cast(out, ctypes.c_void_p)) == 3 and list(out) == [0, 0]
    assert lib.bc_debug_selftest(1, None) == 3
