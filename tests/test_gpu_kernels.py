"""Kernel-level parity on the MI355X: every HIP kernel of libbigcodec_hip.so against the CPU oracle
(the reference's own torch CPU arithmetic) on seeded inputs, through the C ABI."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from audiotokenization_amd import _lib as L
from audiotokenization_amd import blocks as BL
from audiotokenization_amd import conv as CV
from audiotokenization_amd import modules as M
from helpers import assert_close_rel
from oracle import bigcodec_oracle as O
from oracle import vq_c

pytestmark = pytest.mark.gpu


def _rand_wn_conv(m, g, transposed=False):
    with torch.no_grad():
        conv = m.conv if hasattr(m, "conv") and not isinstance(m, (CV.Conv1dWN, CV.ConvTranspose1dWN)) else m
        conv.weight_v.copy_(torch.randn(conv.weight_v.shape, generator=g) / np.sqrt(np.prod(conv.weight_v.shape[1:])))
        conv.weight_g.copy_(torch.rand(conv.weight_g.shape, generator=g) + 0.5)
        conv.bias.copy_(torch.randn(conv.bias.shape, generator=g) * 0.1)
    return conv


def _snake(C, g):
    s = M.SnakeBeta(C, alpha_logscale=True)
    with torch.no_grad():
        s.alpha.copy_(torch.rand(C, generator=g) - 0.5)
        s.beta.copy_(torch.rand(C, generator=g) - 0.5)
    return s


CONV_CASES = [
    # Cin, Cout, K, stride, dilation, causal, snake, residual, tanh, B, T
    (1, 48, 7, 1, 1, False, False, False, False, 2, 1000),
    (1, 16, 7, 1, 1, True, False, False, False, 3, 333),
    (48, 48, 7, 1, 3, False, True, False, False, 2, 777),
    (48, 48, 1, 1, 1, False, True, True, False, 2, 777),
    (16, 16, 7, 1, 9, True, True, False, False, 2, 300),
    (32, 32, 7, 1, 9, False, True, False, False, 1, 257),
    (48, 96, 4, 2, 1, False, True, False, False, 2, 1001),
    (64, 128, 8, 4, 1, False, True, False, False, 2, 803),
    (256, 512, 10, 5, 1, True, True, False, False, 1, 605),
    (384, 768, 10, 5, 1, False, True, False, False, 1, 605),
    (192, 192, 7, 1, 9, False, True, False, False, 2, 300),
    (1536, 1024, 3, 1, 1, False, True, False, False, 2, 50),
    (32, 1, 7, 1, 1, False, False, False, True, 2, 500),
    (32, 1, 7, 1, 1, False, True, True, False, 2, 500),
    (20, 36, 5, 1, 2, False, True, True, False, 2, 64),
    (8, 8, 7, 1, 1, False, False, False, False, 1, 3),
]


@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: "x".join(map(str, c[:5])) + ("c" if c[5] else ""))
def test_conv1d(dev, case, prec):
    Cin, Cout, K, s, d, causal, use_snake, use_res, use_tanh, B, T = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    pad = 0 if causal else (K // 2 * d if s == 1 else s // 2 + s % 2)
    m = CV.WNConv1d(Cin, Cout, kernel_size=K, stride=s, dilation=d, padding=pad, causal=causal)
    conv = _rand_wn_conv(m, g)
    x = torch.randn(B, Cin, T, generator=g)
    snake = _snake(Cout, g) if use_snake else None  # the NEXT Activation1d, fused in the epilogue
    # CPU reference (oracle leaf ops)
    sd = {("conv." if causal else "") + k: v.detach() for k, v in conv.state_dict().items()}
    want = O.conv(x, sd, "", K, s, pad, d, causal)
    res = torch.randn(want.shape, generator=g) if use_res else None
    if use_res:
        want = res + want
    if use_tanh:
        want = torch.tanh(want)
    m.to(dev)
    tol = 3e-6 * max(1.0, np.sqrt(Cin * K / 64))
    co = snake.to(dev).coeffs(dev) if use_snake else None
    rd = res.to(dev) if use_res else None
    got = m.run(x.to(dev), residual=rd, epilogue=int(use_tanh), out_snake=co)
    torch.cuda.synchronize()
    assert got.shape == want.shape
    if use_snake:
        want_s = O.snake_beta(want, snake.alpha.detach().cpu(), snake.beta.detach().cpu())
        assert_close_rel(got.cpu(), want_s, tol * 4, f"conv+snake {case}")
        raw, act = m.run(x.to(dev), residual=rd, out_snake=co, dual=True)
        torch.cuda.synchronize()
        assert_close_rel(raw.cpu(), want, tol, f"conv dual raw {case}")
        assert torch.equal(act, got)
    else:
        assert_close_rel(got.cpu(), want, tol, f"conv {case}")


@pytest.mark.parametrize("Cin,Cout,K,s,d,T,cfgs", [
    (192, 192, 7, 1, 9, 700, (320, 322)), (384, 384, 7, 1, 3, 515, (320, 322)), (192, 192, 7, 1, 1, 256, (320, 322)),
    (768, 768, 7, 1, 9, 300, (320, 322)), (384, 768, 10, 5, 1, 300, (5320, 5322)),
    (192, 384, 4, 2, 1, 520, (2320, 2322)), (96, 192, 4, 2, 1, 600, (2320, 2322)),
    (96, 192, 4, 2, 1, 2001, (2320, 2322)), (192, 384, 4, 2, 1, 1542, (2320, 2322)),
    (768, 1536, 10, 5, 1, 130, (5320, 5322))])
@pytest.mark.parametrize("tprec", ["h3", "bf16", "x6"])
def test_h3_tiles_8_vs_16_waves(dev, Cin, Cout, K, s, d, T, cfgs, tprec):
    """The 192 x 256 h3 tile with 8 waves of 96 x 64 (cfg 320) and with 16 waves of 96 x 32 (322; the
    phase-decomposed strided convs as 1000 s + tile) stages the same B chunks with the same block scales
    and runs the same per-output MFMA chains: bit-identical outputs, and within the conv tolerance of the
    oracle.  The bf16 planes (cfg - 100) and the x6 planes (cfg - 200: three bf16 planes, the 16-wave tile
    without the A-fragment prefetch) run the same two tiles; in x6 the 8-wave tile (120) is the register-A kernel
    (conv1d_x6ra.hip), bit-identical to the 16-wave one.  Stride 2 also at T = 2001 / 1542 (interior column tiles,
    the odd padding, Tin % 4 != 0: the round-6 16-byte quad staging was checked against these and measured without
    gain, profiles/r06i_stride2_quad_staging_rejected.txt)."""
    old = L.precision_mode()
    L.set_precision(tprec)
    if tprec != "h3":
        cfgs = tuple(c - (100 if tprec == "bf16" else 200) for c in cfgs)
    try:
        g = torch.Generator().manual_seed(Cin * 31 + Cout + d)
        pad = K // 2 * d if s == 1 else s // 2 + s % 2
        m = CV.WNConv1d(Cin, Cout, kernel_size=K, stride=s, dilation=d, padding=pad)
        conv = _rand_wn_conv(m, g)
        B = 2
        x = torch.randn(B, Cin, T, generator=g)
        sd = {k: v.detach() for k, v in conv.state_dict().items()}
        want = O.conv(x, sd, "", K, s, pad, d, False)
        Tout = want.shape[-1]
        m.to(dev)
        xd = x.to(dev)
        st = torch.cuda.current_stream().cuda_stream
        outs = {}
        for cfg in cfgs:
            wp, bias = m.packed_as(cfg, dev)
            y = torch.empty(B, Cout, Tout, device=dev)
            L.call("bc_conv1d_fwd", xd.data_ptr(), wp.data_ptr(), L.ptr(bias), 0, 0, 0, y.data_ptr(), 0,
                   B, Cin, T, Cout, Tout, K, s, d, pad, 0, cfg, st)
            torch.cuda.synchronize()
            outs[cfg] = y.cpu()
        tol = 3e-6 * max(1.0, np.sqrt(Cin * K / 64)) if tprec != "bf16" else 2e-2
        assert_close_rel(outs[cfgs[0]], want, tol, f"{tprec} {cfgs[0]}")
        for c in cfgs[1:]:
            assert torch.equal(outs[c], outs[cfgs[0]]), (c, (outs[c] - outs[cfgs[0]]).abs().max())
    finally:
        L._mode = old


@pytest.mark.parametrize("Cin,Cout,d,B,T,cfgs", [(192, 192, 3, 2, 70000, (322, 320)), (384, 384, 9, 3, 24000, (322, 320)),
                                             (768, 768, 9, 3, 8000, (322, 321)), (192, 192, 1, 2, 70000, (222, 220)),
                                             (192, 192, 9, 2, 70000, (122, 120)), (384, 384, 3, 3, 24001, (122, 120)),
                                             (768, 768, 1, 3, 8000, (122, 120))])
def test_k7_tiles_large(dev, Cin, Cout, d, B, T, cfgs):
    """k7 convs at encoder scale (hundreds of tiles, several per CU): two tiles (16 waves and 8 waves, each a
    different grid and tile walk) agree bit for bit, and the output matches the fp64 oracle in windows at the
    start, across tile boundaries and at the end.  x6 (cfg 1xx): the 8-wave 192 x 256 tile is the register-A kernel
    (conv1d_x6ra.hip: weight fragments streamed into registers, the B tile double-buffered; T = 24001 runs its
    single-float staging)."""
    prec = {1: "x6", 2: "bf16", 3: "h3"}[cfgs[0] // 100]
    old = L.precision_mode()
    L.set_precision(prec)
    try:
        g = torch.Generator().manual_seed(Cin + d * 7 + T)
        K, pad = 7, 3 * d
        m = CV.WNConv1d(Cin, Cout, kernel_size=K, dilation=d, padding=pad)
        conv = _rand_wn_conv(m, g)
        x = torch.randn(B, Cin, T, generator=g)
        sd = {k: v.detach() for k, v in conv.state_dict().items()}
        m.to(dev)
        xd = x.to(dev)
        st = torch.cuda.current_stream().cuda_stream
        outs = {}
        for cfg in cfgs:
            wp, bias = m.packed_as(cfg, dev)
            y = torch.empty(B, Cout, T, device=dev)
            L.call("bc_conv1d_fwd", xd.data_ptr(), wp.data_ptr(), L.ptr(bias), 0, 0, 0, y.data_ptr(), 0,
                   B, Cin, T, Cout, T, K, 1, d, pad, 0, cfg, st)
            torch.cuda.synchronize()
            outs[cfg] = y.cpu()
    finally:
        L._mode = old
    assert torch.equal(outs[cfgs[0]], outs[cfgs[1]]), (outs[cfgs[0]] - outs[cfgs[1]]).abs().max()
    got = outs[cfgs[0]]
    tol = 3e-6 * max(1.0, np.sqrt(Cin * K / 64)) if prec != "bf16" else 2e-2
    xp = torch.nn.functional.pad(x.double(), (pad, pad))
    sd64 = {k: v.double() for k, v in sd.items()}
    W = 300
    for s0 in (0, 250, T // 2 - 7, T - W):
        want = O.conv(xp[..., s0:s0 + W + 6 * d], sd64, "", K, 1, 0, d, False)
        assert_close_rel(got[..., s0:s0 + W].double(), want, tol, f"{prec} cfg {cfgs[0]} window {s0}")


CONVT_CASES = [
    # Cin, Cout, stride, causal, snake, B, T
    (64, 32, 2, False, True, 2, 301),
    (96, 48, 5, False, True, 2, 123),
    (40, 20, 4, False, False, 1, 77),
    (32, 16, 2, True, True, 2, 50),
    (48, 24, 5, True, True, 1, 41),
    (1536, 768, 5, False, True, 1, 30),
    (16, 8, 1, False, True, 2, 19),
]


@pytest.mark.parametrize("case", CONVT_CASES, ids=lambda c: "x".join(map(str, c[:3])) + ("c" if c[3] else ""))
def test_conv_transpose1d(dev, case, prec):
    Cin, Cout, s, causal, use_snake, B, T = case
    g = torch.Generator().manual_seed(7 + s)
    K = 2 * s if s != 1 else 1
    kw = {} if causal else {"padding": s // 2 + s % 2 if s != 1 else 0, "output_padding": s % 2 if s != 1 else 0}
    m = CV.WNConvTranspose1d(Cin, Cout, kernel_size=K, stride=s, causal=causal, **kw)
    conv = _rand_wn_conv(m, g)
    x = torch.randn(B, Cin, T, generator=g)
    snake = _snake(Cout, g) if use_snake else None
    sd = {("conv." if causal else "") + k: v.detach() for k, v in conv.state_dict().items()}
    if s == 1:
        want = F.conv_transpose1d(x, O.wn_weight(sd, ""), sd["bias"], 1, 0, 0)
    else:
        want = O.conv_transpose(x, sd, "", s, causal)
    m.to(dev)
    got = m.run(x.to(dev))
    torch.cuda.synchronize()
    assert got.shape == want.shape
    assert_close_rel(got.cpu(), want, 1e-5, f"convT {case}")
    # the op runs bc_convT1d_fwd_ws (contiguous phase rows + interleave); the strided-store bc_convT1d_fwd computes
    # the same phases with the same kernels: bit-identical
    inner = m.conv if hasattr(m, "conv") and isinstance(m.conv, CV.ConvTranspose1dWN) else m
    _, wptrs, bias, cfg = inner.prepared(dev)
    xd = x.to(dev)
    ref = torch.empty_like(got)
    L.call("bc_convT1d_fwd", xd.data_ptr(), wptrs, L.ptr(bias), 0, 0, ref.data_ptr(), 0, B, Cin, T, Cout,
           got.shape[-1], inner.kernel_size, inner.stride, inner.padding, cfg, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(ref, got), (ref - got).abs().max()
    if use_snake:
        co = snake.to(dev).coeffs(dev)
        raw, act = m.run(x.to(dev), out_snake=co, dual=True)
        torch.cuda.synchronize()
        assert torch.equal(raw, got)
        want_s = O.snake_beta(want, snake.alpha.detach().cpu(), snake.beta.detach().cpu())
        assert_close_rel(act.cpu(), want_s, 4e-5, f"convT snake {case}")


@pytest.mark.parametrize("scale", [3.0, 300.0, 20000.0, 1e6])
def test_snake(dev, scale):
    """SnakeBeta against the torch CPU expression and an fp64 evaluation, from small to huge
    arguments (|x*alpha| >= 39000 takes the sinf fallback)."""
    g = torch.Generator().manual_seed(3)
    s = _snake(24, g)
    x = torch.randn(3, 24, 1001, generator=g) * scale
    want = O.snake_beta(x, s.alpha.detach(), s.beta.detach())
    got = s.to(dev)(x.to(dev)).cpu()
    a = torch.exp(s.alpha.detach().cpu().double())[None, :, None]
    ib = (1.0 / (torch.exp(s.beta.detach().cpu()) + 1e-9)).double()[None, :, None]
    t = (x.double() * a.float().double())  # the fp32 product, as the kernel forms it
    t = (x * a.float()).double()
    exact = x.double() + ib * torch.sin(t) ** 2
    ulp = torch.finfo(torch.float32).eps * exact.abs().clamp_min(1e-30)
    err_ulps = ((got.double() - exact).abs() / ulp).max().item()
    cpu_ulps = ((want.double() - exact).abs() / ulp).max().item()
    assert err_ulps <= max(8.0, 2 * cpu_ulps), (err_ulps, cpu_ulps)
    assert_close_rel(got, want, 2e-6, "snake")


def test_aa_activation(dev, golden):
    gd = golden("aa_activation.npz")
    for T in (1, 5, 37, 600):
        act = M.Activation1d(M.SnakeBeta(6, alpha_logscale=True), antialias=True)
        with torch.no_grad():
            act.act.alpha.copy_(torch.from_numpy(gd[f"alpha_{T}"]))
            act.act.beta.copy_(torch.from_numpy(gd[f"beta_{T}"]))
        got = act.to(dev)(torch.from_numpy(gd[f"x_{T}"]).to(dev)).cpu()
        assert_close_rel(got, torch.from_numpy(gd[f"y_{T}"]), 2e-6, f"aa T={T}")


def test_aa_activation_ratios(dev, golden):
    """Activation1d with non-default up / down ratios and tap counts (bc_aa_snake_fwd_ex's general
    kernel) against the reference's outputs (tests/golden/aa_activation_ratios.npz)."""
    gd = golden("aa_activation_ratios.npz")
    meta = gd["meta"]
    for ci, (ru, rd, ku, kd) in enumerate(meta["cases"]):
        for T in meta["T"]:
            k = f"c{ci}_T{T}"
            act = M.Activation1d(M.SnakeBeta(5, alpha_logscale=True), antialias=True, up_ratio=ru, down_ratio=rd,
                                 up_kernel_size=ku, down_kernel_size=kd)
            with torch.no_grad():
                act.act.alpha.copy_(torch.from_numpy(gd[f"alpha_{k}"]))
                act.act.beta.copy_(torch.from_numpy(gd[f"beta_{k}"]))
            want = torch.from_numpy(gd[f"y_{k}"])
            got = act.to(dev)(torch.from_numpy(gd[f"x_{k}"]).to(dev)).cpu()
            assert got.shape == want.shape, (k, got.shape, want.shape)
            assert_close_rel(got, want, 2e-6, f"aa ratios {(ru, rd, ku, kd)} T={T}")


@pytest.mark.parametrize("H,layers,B,T", [(64, 2, 3, 50), (512, 1, 2, 20), (128, 2, 70, 9), (1536, 2, 2, 6),
                                          (256, 2, 130, 7), (512, 2, 64, 40), (1536, 1, 64, 25)])
def test_reslstm(dev, H, layers, B, T, prec):
    """x6 mode with H in {256, 512, 1024, 1536} runs the persistent kernel (lstm_seq.hip), including
    batch slicing (B = 130 -> 3 launches per layer); bc_lstm_status must report no timed-out wait."""
    g = torch.Generator().manual_seed(H + T)
    m = BL.ResLSTM(H, num_layers=layers)
    with torch.no_grad():
        for p in m.lstm.parameters():
            p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) / np.sqrt(H))
    x = torch.randn(B, H, T, generator=g)
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    want = O.res_lstm(x, sd, "", layers)
    got = m.to(dev)(x.to(dev)).cpu()
    assert_close_rel(got, want, 2e-5, f"lstm H={H}")
    # fused output Snake (the Activation1d after the ResLSTM)
    snake = _snake(H, g).to(dev)
    got_s = m.run(x.to(dev), out_snake=snake.coeffs(dev)).cpu()
    want_s = O.snake_beta(want, snake.alpha.detach().cpu(), snake.beta.detach().cpu())
    assert_close_rel(got_s, want_s, 5e-5, f"lstm+snake H={H}")
    assert L.load().bc_lstm_status(1) == 0


@pytest.mark.parametrize("prec", ["h3", "x6"])
@pytest.mark.parametrize("H,B,T", [(1536, 3, 100), (768, 2, 700), (1536, 64, 40), (768, 3, 33)])
def test_lstm_projection_presplit_bit_identical(dev, H, B, T, prec):
    """The ResLSTM input projection on the pre-split GEMM (pw_presplit.hip: B planes (and, h3, block scales) made once
    per 256-column tile, copied by LDS-DMA; x6 on 128-row tiles over the cfg-122 weights) against the same projection
    on conv1d_x6_kernel cfg 322 / 122: the same blocks, scales and MFMA chains, so the layer outputs are
    bit-identical; T * B not a multiple of 256 (ragged last column tile) and not a multiple of 4 (no 16-byte rows)
    included; and within the oracle's tolerance."""
    old = L.precision_mode()
    L.set_precision(prec)
    lib = L.load()
    try:
        g = torch.Generator().manual_seed(H * 3 + B + T)
        m = BL.ResLSTM(H, num_layers=2)
        with torch.no_grad():
            for p in m.lstm.parameters():
                p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) / np.sqrt(H))
        x = torch.randn(B, H, T, generator=g) * torch.exp(torch.randn(1, H, 1, generator=g))
        sd = {k: v.detach() for k, v in m.state_dict().items()}
        m.to(dev)
        xd = x.to(dev)
        prev = lib.bc_debug_set_lstm_presplit(2)  # the pre-split GEMM at any size (below 32 column tiles too)
        y_ps = m(xd).cpu()
        lib.bc_debug_set_lstm_presplit(0)
        y_x6 = m(xd).cpu()
        lib.bc_debug_set_lstm_presplit(prev)
        assert lib.bc_lstm_status(1) == 0
    finally:
        L._mode = old
    assert torch.equal(y_ps, y_x6), (y_ps - y_x6).abs().max()
    want = O.res_lstm(x, sd, "", 2)
    assert_close_rel(y_ps, want, 2e-5, f"lstm {prec} presplit H={H}")


@pytest.mark.parametrize("lprec", ["h3", "x6"])
def test_reslstm_half_split_bit_identical(dev, lprec):
    """The persistent recurrence runs a launch of <= 32 clips as two halves of 16 (NTH = 1; half 1 empty at <= 16 clips)
    and a launch of 33-64 clips as two halves of 32: a clip's gates are summed over the same K ranges, waves and MFMA chains either way,
    so in x6 (exact per-element operand splits everywhere) the first 32 / 20 clips of a 64-clip batch come out
    bit-identical when run alone.  In h3 the input projection's block scales span the clips of a column tile, so
    there only agreement at the 22-bit operand level is asserted; both match the oracle."""
    old = L.precision_mode()
    L.set_precision(lprec)
    try:
        H, T = 1536, 40
        g = torch.Generator().manual_seed(1536 + T)
        m = BL.ResLSTM(H, num_layers=2)
        with torch.no_grad():
            for p in m.lstm.parameters():
                p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) / np.sqrt(H))
        x = torch.randn(64, H, T, generator=g)
        sd = {k: v.detach() for k, v in m.state_dict().items()}
        m.to(dev)
        xd = x.to(dev)
        full = m(xd).cpu()
        y32 = m(xd[:32].contiguous()).cpu()
        y20 = m(xd[:20].contiguous()).cpu()
        # <= 16 clips: half 1 is empty (its chain still runs and hides half 0's hand-off latency)
        small = {n: m(xd[:n].contiguous()).cpu() for n in (16, 5, 1)}
        assert L.load().bc_lstm_status(1) == 0
    finally:
        L._mode = old
    if lprec == "x6":
        assert torch.equal(y32, full[:32]), (y32 - full[:32]).abs().max()
        assert torch.equal(y20, full[:20]), (y20 - full[:20]).abs().max()
        for n, y in small.items():
            assert torch.equal(y, full[:n]), (n, (y - full[:n]).abs().max())
    else:
        assert_close_rel(y32, full[:32], 2e-6, "h3 lstm 32 vs 64 clips")
        assert_close_rel(y20, full[:20], 2e-6, "h3 lstm 20 vs 64 clips")
        for n, y in small.items():
            assert_close_rel(y, full[:n], 2e-6, f"h3 lstm {n} vs 64 clips")
    want = O.res_lstm(x[:20], sd, "", 2)
    assert_close_rel(y20, want, 2e-5, f"lstm {lprec} 20 clips")


@pytest.mark.parametrize("Cin,Cout,K,d", [(384, 384, 7, 9), (1536, 1024, 3, 1), (96, 96, 7, 1), (768, 768, 1, 1)])
def test_x6_error_vs_fp64(dev, Cin, Cout, K, d):
    """The 3xbf16-split MFMA conv is fp32-accurate: its error against an fp64 evaluation is no larger
    than (1.25x) the native fp32 MFMA kernel's, measured as max |y - y64| / max(sum |w x|).  The
    2xfp16 block-scaled split ("h3", 22-bit operands) stays within 2x of it."""
    g = torch.Generator().manual_seed(Cin + K)
    m = CV.WNConv1d(Cin, Cout, kernel_size=K, dilation=d, padding=K // 2 * d)
    conv = _rand_wn_conv(m, g)
    x = torch.randn(2, Cin, 300, generator=g) * torch.exp(torch.randn(1, Cin, 1, generator=g))
    sd = {k: v.detach() for k, v in conv.state_dict().items()}
    w = O.wn_weight(sd, "").double()
    y64 = F.conv1d(x.double(), w, sd["bias"].double(), 1, K // 2 * d, d)
    scale = F.conv1d(x.double().abs(), w.abs(), None, 1, K // 2 * d, d).max()
    m.to(dev)
    errs = {}
    old = L.precision_mode()
    try:
        for p in ("fp32", "x6", "h3"):
            L.set_precision(p)
            y = m.run(x.to(dev)).cpu().double()
            errs[p] = float((y - y64).abs().max() / scale)
    finally:
        L._mode = old
    print(f"conv {Cin}->{Cout} k{K} d{d}: max|y - y64| / max(sum|w x|): fp32 MFMA {errs['fp32']:.3e}, "
          f"x6 {errs['x6']:.3e}, h3 {errs['h3']:.3e}")
    assert errs["x6"] <= 1.25 * errs["fp32"] + 1e-9, errs
    assert errs["h3"] <= 2.0 * errs["fp32"] + 1e-9, errs
    assert errs["fp32"] < 1e-6, errs


@pytest.mark.parametrize("Cin,K,pw", [(96, 7, False), (256, 1, True), (160, 3, False)])
def test_h3_block_scaling(dev, Cin, K, pw):
    """h3 block scaling: channel groups whose magnitudes span 1e-30 .. 1e30 (beyond fp16's range in
    both directions; chunks of 32 channels that grow and shrink, so the per-chunk scale changes and the
    accumulator is rescaled) and all-zero chunks.  Each output's error against fp64 stays at the fp32
    level of its own |w||x| scale."""
    g = torch.Generator().manual_seed(Cin * 3 + K)
    Cout = 64
    m = CV.WNConv1d(Cin, Cout, kernel_size=K, padding=K // 2)
    conv = _rand_wn_conv(m, g)
    mags = torch.tensor([1e-30, 1.0, 1e30, 0.0, 1e-3, 1e12, 1e-12, 7.0])
    grp = mags[(torch.arange(Cin) // 32) % len(mags)].view(1, Cin, 1)
    x = torch.randn(2, Cin, 260, generator=g) * grp
    sd = {k: v.detach() for k, v in conv.state_dict().items()}
    w = O.wn_weight(sd, "").double()
    y64 = F.conv1d(x.double(), w, sd["bias"].double(), 1, K // 2, 1)
    scale = F.conv1d(x.double().abs(), w.abs(), None, 1, K // 2, 1) + sd["bias"].double().abs().view(1, -1, 1)
    m.to(dev)
    old = L.precision_mode()
    try:
        L.set_precision("h3")
        y = m.run(x.to(dev)).cpu().double()
    finally:
        L._mode = old
    assert torch.isfinite(y).all()
    rel = ((y - y64).abs() / scale).max().item()
    print(f"h3 block scaling Cin={Cin} K={K}: max |y - y64| / (sum|w x| + |b|) = {rel:.3e}")
    assert rel < 2e-6, rel


@pytest.mark.parametrize("C,d,causal,B,T", [(48, 1, False, 2, 1001), (48, 9, False, 1, 700), (96, 3, False, 2, 513),
                                           (48, 3, False, 1, 24000), (48, 1, False, 3, 4096), (48, 9, True, 2, 777),
                                           (64, 9, False, 2, 300), (16, 3, True, 2, 257), (64, 1, False, 1, 260),
                                           (96, 9, True, 1, 999), (32, 1, False, 3, 64)])
@pytest.mark.parametrize("ru_prec", ["x6", "h3"])
def test_resunit_fused(dev, C, d, causal, B, T, ru_prec):
    """bc_resunit_fwd (one launch per ResidualUnit, x6 or h3) against the oracle: plain output, and the
    dual raw + next-Snake output the encoder flow uses."""
    old = L.precision_mode()
    L.set_precision(ru_prec)
    try:
        g = torch.Generator().manual_seed(C * 10 + d)
        ru = BL.ResidualUnit(C, dilation=d, causal=causal)
        _rand_wn_conv(ru.block[1], g)
        _rand_wn_conv(ru.block[3], g)
        for k in (0, 2):
            s = _snake(C, g)
            ru.block[k].act.load_state_dict(s.state_dict())
        nxt = M.Activation1d(activation=_snake(C, g))
        x = torch.randn(B, C, T, generator=g)
        sd = {k: v.detach() for k, v in ru.state_dict().items()}
        want = O.residual_unit(x, sd, "", d, causal, False)
        want_s = O.snake_beta(want, nxt.act.alpha.detach(), nxt.act.beta.detach())
        ru.to(dev)
        nxt.to(dev)
        assert ru._fused_cfg() >= 0
        xd = x.to(dev)
        xa = ru.first_act(xd)
        got = ru.flow(xd, xa)[0].cpu()
        raw, act = ru.flow(xd, xa, want_raw=True, next_act=nxt)
        _, act_only = ru.flow(xd, xa, want_raw=False, next_act=nxt)
        # snake on load (bc_resunit_fwd_snake_in): the first Snake applied while staging the raw input
        # computes the same operations in the same order as the producer epilogue -> bit-identical
        assert ru.snake_on_load()
        lazy = ru.flow(xd, None)[0].cpu()
        lraw, lact = ru.flow(xd, None, want_raw=True, next_act=nxt)
    finally:
        L._mode = old
    assert_close_rel(got, want, 2e-5, f"resunit C={C} d={d}")
    assert torch.equal(raw.cpu(), got)
    assert_close_rel(act.cpu(), want_s, 5e-5, "resunit + next snake")
    assert torch.equal(act_only.cpu(), act.cpu())
    assert torch.equal(lazy, got)
    assert torch.equal(lraw.cpu(), got) and torch.equal(lact.cpu(), act.cpu())


@pytest.mark.parametrize("d,causal,B,T", [(1, False, 2, 1001), (3, False, 1, 24000), (9, False, 1, 24000),
                                         (9, True, 2, 6000), (3, True, 1, 513), (1, False, 3, 256), (9, False, 2, 130),
                                         (3, False, 2, 1001)])
def test_resunit_w16_c192(dev, d, causal, B, T):
    """The one-launch x6 ResidualUnit at C = 192 (resunit_w16.hip: the k7 main loop of the 16-wave tile, h through LDS,
    k=1 weights streamed into registers) against the oracle, against the two-launch x6 path (k7 conv writing h, k=1
    conv reading it: the same splits and the same per-output MFMA chains, so equal to fp32 rounding at most), with the
    dual raw + next-Snake output, and snake on load (the producer writes only the raw tensor) bit-identical to a
    producer-side Snake.  T = 1001 / 513 / 130 take the single-float staging (Tin % 4 != 0), the others the 16-byte one;
    T = 130 / 256 / 513 leave partial 256-column tiles."""
    from audiotokenization_amd.blocks import produce_conv

    old = L.precision_mode()
    L.set_precision("x6")
    try:
        g = torch.Generator().manual_seed(1920 + d * 7 + T)
        ru = BL.ResidualUnit(192, dilation=d, causal=causal)
        _rand_wn_conv(ru.block[1], g)
        _rand_wn_conv(ru.block[3], g)
        for k in (0, 2):
            ru.block[k].act.load_state_dict(_snake(192, g).state_dict())
        nxt = M.Activation1d(activation=_snake(192, g))
        x = torch.randn(B, 192, T, generator=g)
        sd = {k: v.detach() for k, v in ru.state_dict().items()}
        want = O.residual_unit(x, sd, "", d, causal, False)
        want_s = O.snake_beta(want, nxt.act.alpha.detach(), nxt.act.beta.detach())
        ru.to(dev)
        nxt.to(dev)
        cfg = ru._fused_cfg()
        name = L.resunit_kernel_name(cfg, 192, d)
        assert cfg == 122 and name.startswith("resunit_w16_kernel<3, "), (cfg, name)
        xd = x.to(dev)
        xa = ru.first_act(xd)
        got = ru.flow(xd, xa)[0].cpu()
        raw, act = ru.flow(xd, xa, want_raw=True, next_act=nxt)
        _, act_only = ru.flow(xd, xa, want_raw=False, next_act=nxt)
        assert ru.snake_on_load()
        lazy = ru.flow(xd, None)[0].cpu()
        lraw, lact = ru.flow(xd, None, want_raw=True, next_act=nxt)
        _, h = produce_conv(ru.block[1], xa, None, want_raw=False, next_act=ru.block[2])
        two = produce_conv(ru.block[3], h, residual=xd, want_raw=True, next_act=None)[0].cpu()
    finally:
        L._mode = old
    diff = (got - two).abs().max().item()
    print(f"w16 C=192 d={d} causal={causal} B={B} T={T}: fused vs two launches max |d| {diff:.3e}"
          f" ({'bit-identical' if diff == 0 else 'not bit-identical'})")
    assert_close_rel(got, want, 2e-5, f"w16 resunit d={d} T={T}")
    assert_close_rel(got, two, 2e-6, f"w16 resunit d={d}: one launch vs two")
    assert torch.equal(raw.cpu(), got)
    assert_close_rel(act.cpu(), want_s, 5e-5, "w16 resunit + next snake")
    assert torch.equal(act_only.cpu(), act.cpu())
    assert torch.equal(lazy, got)
    assert torch.equal(lraw.cpu(), got) and torch.equal(lact.cpu(), act.cpu())


@pytest.mark.parametrize("C,d,causal,B,T", [(48, 1, False, 2, 1001), (48, 9, True, 1, 24000), (96, 3, False, 2, 513),
                                           (96, 9, False, 1, 4096), (64, 1, True, 2, 300), (16, 3, False, 3, 257),
                                           (192, 1, False, 2, 1001), (192, 9, True, 1, 24000), (192, 3, False, 2, 130)])
def test_resunit_fused_bf16(dev, C, d, causal, B, T):
    """Precision 'bf16' (config 5) runs the ResidualUnit in one launch too (resunit_x6_kernel<..., P = 1>):
    the k=7 input and the activated h rounded to bf16 as the lone bf16 convs round their inputs, fp32
    accumulation.  Against the two-launch bf16 path: the same roundings and the same accumulation
    order, so agreement to a few fp32 ulps; against the fp32 oracle: bf16-rounding sized.  C = 192 runs the
    16-wave unit (resunit_w16_kernel<1, ...>: phase 1 four taps per K-step, h rounded to bf16 in LDS)."""
    from audiotokenization_amd.blocks import produce_conv

    old = L.precision_mode()
    L.set_precision("bf16")
    try:
        g = torch.Generator().manual_seed(C * 10 + d + 7)
        ru = BL.ResidualUnit(C, dilation=d, causal=causal)
        _rand_wn_conv(ru.block[1], g)
        _rand_wn_conv(ru.block[3], g)
        for k in (0, 2):
            ru.block[k].act.load_state_dict(_snake(C, g).state_dict())
        x = torch.randn(B, C, T, generator=g)
        sd = {k: v.detach() for k, v in ru.state_dict().items()}
        want = O.residual_unit(x, sd, "", d, causal, False)
        ru.to(dev)
        cfg = ru._fused_cfg()
        assert 200 <= cfg < 300, cfg
        name = L.resunit_kernel_name(cfg, C, d)
        if C == 192:
            assert cfg == 222 and name.startswith("resunit_w16_kernel<1, "), (cfg, name)
        else:
            assert "resunit_x6_kernel" in name and ", 1, " in name, name
        xd = x.to(dev)
        xa = ru.first_act(xd)
        got = ru.flow(xd, xa)[0].cpu()
        lazy = ru.flow(xd, None)[0].cpu()
        _, h = produce_conv(ru.block[1], xa, None, want_raw=False, next_act=ru.block[2])
        two = produce_conv(ru.block[3], h, residual=xd, want_raw=True, next_act=None)[0].cpu()
    finally:
        L._mode = old
    assert torch.equal(lazy, got)
    assert_close_rel(got, two, 1e-5, f"bf16 resunit C={C} d={d}: one launch vs two")
    assert_close_rel(got, want, 2e-2, f"bf16 resunit C={C} d={d} vs fp32 oracle")
    rel = ((got - want).abs().max() / want.abs().max()).item()
    assert rel > 1e-5, rel  # really bf16 products


@pytest.mark.parametrize("prec,C,alt", [("h3", 96, 309), ("bf16", 96, 209), ("x6", 96, 123), ("bf16", 48, 224),
                                        ("bf16", 48, 206)])
@pytest.mark.parametrize("d,B,T", [(1, 2, 1001), (9, 1, 4096), (3, 1, 129)])
def test_resunit_tiles_bit_identical(dev, prec, C, alt, d, B, T):
    """The one-launch ResidualUnit on another tile shape (123, the h3 / bf16 default at C = 96: 96 x 128 as 2 x 4 waves of
    48 x 32, against 109's 8 waves of 96 x 16; 124 / 106: 48 x 512 /
    48 x 256, 48 x 64 / 48 x 32 per wave) computes every output with the same per-output MFMA chain, the same staged
    columns per chunk (h3 block scales) and the same h tile: bit-identical to the default tile, and within the
    oracle's tolerance."""
    old = L.precision_mode()
    L.set_precision(prec)
    try:
        g = torch.Generator().manual_seed(C + 13 * d + T)
        ru = BL.ResidualUnit(C, dilation=d)
        _rand_wn_conv(ru.block[1], g)
        _rand_wn_conv(ru.block[3], g)
        for k in (0, 2):
            ru.block[k].act.load_state_dict(_snake(C, g).state_dict())
        nxt = M.Activation1d(activation=_snake(C, g))
        x = torch.randn(B, C, T, generator=g)
        sd = {k: v.detach() for k, v in ru.state_dict().items()}
        want = O.residual_unit(x, sd, "", d, False, False)
        ru.to(dev)
        nxt.to(dev)
        xd = x.to(dev)
        base = ru._fused_cfg()
        assert base != alt
        if prec == "h3" and C == 48:
            pytest.skip("C = 48 h3 runs the strip kernel")
        ref_raw, ref_act = ru._flow_fused(base, xd, None, True, nxt)
        raw, act = ru._flow_fused(alt, xd, None, True, nxt)
        ref_raw, ref_act, raw, act = ref_raw.cpu(), ref_act.cpu(), raw.cpu(), act.cpu()
    finally:
        L._mode = old
    assert torch.equal(raw, ref_raw), f"{prec} C={C} cfg {alt} vs {base}: max |d| {(raw - ref_raw).abs().max().item():.3e}"
    assert torch.equal(act, ref_act)
    assert_close_rel(raw, want, 2e-2 if prec == "bf16" else 2e-5, f"{prec} resunit C={C} d={d} cfg {alt}")


@pytest.mark.parametrize("d,B,T", [(3, 1, 1001), (3, 1, 4096), (1, 1, 24000), (9, 1, 24000), (3, 2, 700),
                                   (2, 1, 1001), (4, 1, 1001), (5, 1, 1001), (9, 2, 129), (1, 3, 128), (3, 1, 5)])
def test_resunit_c48_h3_sweep(dev, d, B, T):
    """The C = 48 units in h3 (the streaming strip kernel at d = 1 / 3 / 9, resunit_rr at other dilations) over
    dilations, clip lengths around the 128-column block and strip boundaries, and batch sizes: against the
    oracle, and snake on load bit-identical to a producer-side Snake (tools/ru_rr_check.py's sweep).
    A failure prints the bad columns / channels."""
    old = L.precision_mode()
    L.set_precision("h3")
    try:
        g = torch.Generator().manual_seed(480 + d * 7 + T)
        ru = BL.ResidualUnit(48, dilation=d)
        _rand_wn_conv(ru.block[1], g)
        _rand_wn_conv(ru.block[3], g)
        for k in (0, 2):
            s_ = _snake(48, g)
            ru.block[k].act.load_state_dict(s_.state_dict())
        nxt = M.Activation1d(activation=_snake(48, g))
        x = torch.randn(B, 48, T, generator=g)
        sd = {k: v.detach() for k, v in ru.state_dict().items()}
        want = O.residual_unit(x, sd, "", d, False, False)
        want_s = O.snake_beta(want, nxt.act.alpha.detach(), nxt.act.beta.detach())
        ru.to(dev)
        nxt.to(dev)
        xd = x.to(dev)
        lazy = ru.flow(xd, None)[0].cpu()
        eager = ru.flow(xd, ru.first_act(xd))[0].cpu()
        lraw, lact = ru.flow(xd, None, want_raw=True, next_act=nxt)
        name = L.resunit_kernel_name(ru._fused_cfg(), 48, d)
    finally:
        L._mode = old
    bad = (lazy - want).abs() > 1e-4 * want.abs().max()
    cols = torch.nonzero(bad.any(1).any(0)).flatten()
    chans = torch.nonzero(bad.any(2).any(0)).flatten()
    print(f"C=48 d={d} B={B} T={T} ({name}): bad cols {cols[:10].tolist()} (n={cols.numel()}), chans {chans[:12].tolist()}")
    assert_close_rel(lazy, want, 2e-5, f"resunit C=48 d={d} T={T}")
    assert torch.equal(lazy, eager)
    assert torch.equal(lraw.cpu(), lazy)
    assert_close_rel(lact.cpu(), want_s, 5e-5, "resunit C=48 + next snake")


@pytest.mark.parametrize("d", [1, 9])
def test_resunit_strip_long_clip(dev, d):
    """The h3 C = 48 strip kernel on ONE clip of T = 2 200 000 samples (92 s @24 kHz): window starts past 2^21 samples,
    where the interior windows' byte offset (ws * 4) crosses 2^23 -- the scalar-offset range a gfx950 buffer load faulted
    at; the offset now rides in the resource base.  Checked against the oracle in windows (the
    unit is local: output [t0, t1) needs input [t0 - 3d, t1 + 3d)): before 2^21, across it, near 2^22 * 0.5 + T / 2, and
    the clip's end (the real zero padding)."""
    T = 2_200_000
    old = L.precision_mode()
    L.set_precision("h3")
    try:
        g = torch.Generator().manual_seed(4821 + d)
        ru = BL.ResidualUnit(48, dilation=d)
        _rand_wn_conv(ru.block[1], g)
        _rand_wn_conv(ru.block[3], g)
        for k in (0, 2):
            ru.block[k].act.load_state_dict(_snake(48, g).state_dict())
        x = torch.randn(1, 48, T, generator=g)
        sd = {k: v.detach() for k, v in ru.state_dict().items()}
        ru.to(dev)
        name = L.resunit_kernel_name(ru._fused_cfg(), 48, d)
        assert name == f"resunit_strip_kernel<{d}>", name
        got = ru.flow(x.to(dev), None)[0].cpu()
        torch.cuda.synchronize()
    finally:
        L._mode = old
    h = 3 * d
    for t0 in (1000, 2_097_000, 2_150_000, T - 3000):
        t1 = min(t0 + 3000, T)
        lo, hi = max(t0 - h, 0), min(t1 + h, T)
        want = O.residual_unit(x[..., lo:hi], sd, "", d, False, False)[..., t0 - lo:t0 - lo + (t1 - t0)]
        assert_close_rel(got[..., t0:t1], want, 2e-5, f"strip d={d} T={T} window {t0}")


@pytest.mark.parametrize("Cin,Cout,K,s,d", [(384, 384, 7, 1, 9), (48, 96, 4, 2, 1), (768, 768, 1, 1, 1)])
def test_bf16_precision_error(dev, Cin, Cout, K, s, d):
    """precision 'bf16' (config 5): one bf16 product per pair, fp32 accumulation.  Its error against
    fp64 is bf16-rounding sized: well below 2^-7 of the |w||x| scale, and far above the x6 path's."""
    g = torch.Generator().manual_seed(Cin * K)
    pad = K // 2 * d if s == 1 else s // 2 + s % 2
    m = CV.WNConv1d(Cin, Cout, kernel_size=K, stride=s, dilation=d, padding=pad)
    conv = _rand_wn_conv(m, g)
    x = torch.randn(2, Cin, 400, generator=g)
    sd = {k: v.detach() for k, v in conv.state_dict().items()}
    w = O.wn_weight(sd, "").double()
    y64 = F.conv1d(x.double(), w, sd["bias"].double(), s, pad, d)
    scale = F.conv1d(x.double().abs(), w.abs(), None, s, pad, d).max()
    m.to(dev)
    errs = {}
    old = L.precision_mode()
    try:
        for p in ("x6", "bf16"):
            L.set_precision(p)
            y = m.run(x.to(dev)).cpu().double()
            errs[p] = float((y - y64).abs().max() / scale)
    finally:
        L._mode = old
    print(f"conv {Cin}->{Cout} k{K} s{s} d{d}: relative error x6 {errs['x6']:.3e}, bf16 {errs['bf16']:.3e}")
    assert errs["bf16"] < 2 ** -7, errs
    assert errs["bf16"] > 50 * errs["x6"], errs  # really computed with bf16 products


def test_vq_argmin_bit_exact(dev, golden):
    """Given the same projected latents z_e, the HIP search returns the reference's indices
    exactly, including the planted exact ties (lowest index wins) and zero / tiny rows."""
    gd = golden("vq_decode_latents.npz")
    lib = L.load()
    cb = torch.from_numpy(gd["codebook"]).to(dev)
    cbn = torch.empty_like(cb)
    csq = torch.empty(cb.shape[0], device=dev)
    st = torch.cuda.current_stream().cuda_stream
    L.check(lib.bc_vq_prepare_codebook(cb.data_ptr(), cbn.data_ptr(), csq.data_ptr(), cb.shape[0], 8, st), "prep")
    cbn_c, csq_c = vq_c.prepare(gd["codebook"])
    torch.cuda.synchronize()
    assert np.array_equal(cbn.cpu().numpy(), cbn_c) and np.array_equal(csq.cpu().numpy(), csq_c)
    ze = torch.from_numpy(gd["z_e"]).to(dev)
    idx = torch.empty(ze.shape[0], dtype=torch.int64, device=dev)
    L.check(lib.bc_vq_argmin(ze.data_ptr(), cbn.data_ptr(), csq.data_ptr(), idx.data_ptr(), ze.shape[0], 8192, 8,
                             st), "argmin")
    torch.cuda.synchronize()
    assert np.array_equal(idx.cpu().numpy(), gd["indices"])


def test_vq_argmin_random_large(dev):
    """200k random rows: HIP search == C oracle bit for bit."""
    rng = np.random.default_rng(5)
    cbk = (rng.random((8192, 8), dtype=np.float32) * 2 - 1).astype(np.float32)
    ze = (rng.standard_normal((20000, 8)) * rng.lognormal(size=(20000, 1))).astype(np.float32)
    want = vq_c.argmin(ze, cbk)
    fvq = M.FactorizedVectorQuantize(dim=16, codebook_size=8192, codebook_dim=8, commitment=0.25)
    with torch.no_grad():
        fvq._codebook.weight.copy_(torch.from_numpy(cbk))
    fvq.to(dev)
    cb, cbn, csq, *_ = fvq.prepared(dev)
    zt = torch.from_numpy(ze).to(dev)
    idx = torch.empty(ze.shape[0], dtype=torch.int64, device=dev)
    L.call("bc_vq_argmin", zt.data_ptr(), cbn.data_ptr(), csq.data_ptr(), idx.data_ptr(), ze.shape[0], 8192, 8,
           torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(idx.cpu().numpy(), want)


def test_fvq_forward_and_vq2emb(dev):
    g = torch.Generator().manual_seed(11)
    D = 96
    rvq = M.ResidualVQ(num_quantizers=1, dim=D, codebook_size=8192, codebook_dim=8, commitment=0.25)
    with torch.no_grad():
        for p in rvq.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.3)
    rvq.eval()
    z = torch.randn(2, D, 333, generator=g)
    sd = {k: v.detach() for k, v in rvq.state_dict().items()}
    want_q, want_idx, _ = O.rvq_forward(z, sd, "", 1)
    _, _, _, ze = O.fvq_forward(z, sd, "layers.0.", return_ze=True)
    rvq.to(dev)
    got_q, got_idx, loss = rvq(z.to(dev))
    torch.cuda.synchronize()
    # indices: exact except at fp32 near-ties of the in_proj (certified by the C oracle's own gap)
    _, best, second = vq_c.argmin(ze.permute(0, 2, 1).reshape(-1, 8).numpy(), sd["layers.0._codebook.weight"].numpy(),
                                  return_dists=True)
    bad = np.nonzero(got_idx.cpu().numpy().reshape(-1) != want_idx.numpy().reshape(-1))[0]
    assert bad.size <= 2 and np.all((second - best)[bad] < 1e-5)
    ok = np.ones(z.shape[0] * z.shape[2], bool)
    ok[bad] = False
    gq = got_q.cpu().permute(0, 2, 1).reshape(-1, D)[ok]
    wq = want_q.permute(0, 2, 1).reshape(-1, D)[ok]
    assert_close_rel(gq, wq, 1e-5, "post")
    assert loss.shape == (1,) and float(loss.abs().sum()) == 0.0
    # vq2emb on the reference's indices (B, T, Nq) -> (B, T, D)
    vq = want_idx.permute(1, 2, 0).contiguous()
    emb = rvq.vq2emb(vq.to(dev)).cpu()
    want_emb = O.vq2emb(vq, sd, "", 1)
    assert_close_rel(emb, want_emb, 1e-6, "vq2emb")


@pytest.mark.parametrize("nq", [2, 4])
def test_multi_quantizer_rvq(dev, nq):
    """vq_num_quantizers > 1 (residual_vq.py:21-40): each layer quantizes the
    residual the previous ones left.  Indices (nq, B, F) against the oracle: a frame may differ only
    after a certified fp32 near-tie (first differing layer's oracle top-2 gap < 1e-5; later layers then
    see another residual), at most 2 frames; z_q within 1e-5 on the frames that agree; loss (nq,) zeros;
    vq2emb on the oracle's codes within 1e-6."""
    g = torch.Generator().manual_seed(23 + nq)
    D = 96
    rvq = M.ResidualVQ(num_quantizers=nq, dim=D, codebook_size=8192, codebook_dim=8, commitment=0.25)
    with torch.no_grad():
        for p in rvq.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.3)
    rvq.eval()
    z = torch.randn(2, D, 333, generator=g)
    sd = {k: v.detach() for k, v in rvq.state_dict().items()}
    want_q, want_idx, _ = O.rvq_forward(z, sd, "", nq)
    rvq.to(dev)
    got_q, got_idx, loss = rvq(z.to(dev))
    torch.cuda.synchronize()
    assert tuple(got_idx.shape) == (nq, 2, 333) and tuple(loss.shape) == (nq,)
    assert float(loss.abs().sum()) == 0.0
    gi, wi = got_idx.cpu().numpy().reshape(nq, -1), want_idx.numpy().reshape(nq, -1)
    bad = np.nonzero((gi != wi).any(0))[0]
    # certify each differing frame at its first differing layer, on the oracle's own residual there
    res = z.clone()
    gaps = {}
    for q in range(nq):
        pre = f"layers.{q}."
        zq, _, _, ze = O.fvq_forward(res, sd, pre, return_ze=True)
        _, best, second = vq_c.argmin(ze.permute(0, 2, 1).reshape(-1, 8).numpy(),
                                      sd[pre + "_codebook.weight"].numpy(), return_dists=True)
        for f in bad:
            if f not in gaps and gi[q, f] != wi[q, f]:
                gaps[f] = float(second[f] - best[f])
        res = res - zq
    print(f"nq={nq}: {bad.size} differing frames of {gi.shape[1]}, gaps {sorted(gaps.values())}")
    assert bad.size <= 2 and all(v < 1e-5 for v in gaps.values())
    ok = np.ones(gi.shape[1], bool)
    ok[bad] = False
    gq = got_q.cpu().permute(0, 2, 1).reshape(-1, D)[ok]
    wq = want_q.permute(0, 2, 1).reshape(-1, D)[ok]
    assert_close_rel(gq, wq, 1e-5, f"rvq nq={nq} post")
    vq = want_idx.permute(1, 2, 0).contiguous()
    emb = rvq.vq2emb(vq.to(dev)).cpu()
    assert_close_rel(emb, O.vq2emb(vq, sd, "", nq), 1e-6, f"rvq nq={nq} vq2emb")


def test_synth_clips_device_equals_host(dev):
    from audiotokenization_amd import synth
    from audiotokenization_amd.extract import synth_batch

    x = synth_batch(3, 5000, 17, dev).cpu().numpy()[:, 0]
    assert np.array_equal(x, synth.synth_clips(3, 5000, clip0=17))


def test_abi_rejects_bad_args(dev):
    lib = L.load()
    # invalid cfg id, or a phase-decomposed cfg for another stride -> BC_ERR_ARG, nothing launched
    assert lib.bc_conv1d_fwd(1, 1, None, None, None, None, 1, None, 1, 48, 10, 48, 10, 7, 1, 1, 3, 0, 99, None) == 1
    assert lib.bc_conv1d_fwd(1, 1, None, None, None, None, 1, None, 1, 48, 10, 48, 10, 7, 1, 1, 3, 0, 5109, None) == 1
    assert lib.bc_vq_argmin(1, 1, 1, 1, 10, 8192, 4, None) == 3


def test_lstm_timeout_is_loud(dev):
    """a persistent ResLSTM launch whose workgroups give up waiting (forced here with
    a poll limit of 1 through the diagnostic bc_debug_set_lstm_spin_limit) must raise, not return wrong
    latents; the next normal call is correct again."""
    import ctypes

    from audiotokenization_amd import synth
    from helpers import build_models

    lib = L.load()
    setter = lib.bc_debug_set_lstm_spin_limit
    setter.argtypes = [ctypes.c_longlong]
    setter.restype = ctypes.c_int
    enc, dec, *_ = build_models("base", device=dev)
    x = torch.from_numpy(synth.synth_clips(2, 24000, clip0=0)).unsqueeze(1).to(dev)
    with torch.no_grad():
        good = enc(x)
        assert setter(1) == 0
        try:
            with pytest.raises(L.BigCodecLibraryError, match="timed out"):
                enc(x)
        finally:
            assert setter(0) == 0
        again = enc(x)
        torch.cuda.synchronize()
    assert torch.equal(good, again)
    assert lib.bc_lstm_status(1) > 0  # the process-wide diagnostic saw them (reset for later tests)


@pytest.mark.parametrize("D,layers,B,T", [(64, 2, 3, 37), (512, 2, 4, 50), (1536, 1, 2, 23)])
def test_reslstm_bidirectional(dev, D, layers, B, T):
    """ResLSTM(bidirectional=True) (vq/module.py:150-152: nn.LSTM(D, D/2, bidirectional)) against torch's
    own CPU LSTM (oracle.res_lstm): D = 64 runs the per-step kernels (H = 32), D = 512 / 1536 the
    persistent one (H = 256 / 768) for both directions; plus the fused output Snake."""
    L.load().bc_lstm_status(1)
    g = torch.Generator().manual_seed(D + T)
    m = BL.ResLSTM(D, num_layers=layers, bidirectional=True)
    H = D // 2
    with torch.no_grad():
        for p in m.lstm.parameters():
            p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) / np.sqrt(H))
    assert any(k.endswith("_reverse") for k in m.state_dict())  # torch's parameter names (checkpoint keys)
    x = torch.randn(B, D, T, generator=g)
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    want = O.res_lstm(x, sd, "", layers, bidirectional=True)
    got = m.to(dev)(x.to(dev)).cpu()
    assert_close_rel(got, want, 2e-5, f"bidirectional lstm D={D}")
    snake = _snake(D, g).to(dev)
    got_s = m.run(x.to(dev), out_snake=snake.coeffs(dev)).cpu()
    want_s = O.snake_beta(want, snake.alpha.detach().cpu(), snake.beta.detach().cpu())
    assert_close_rel(got_s, want_s, 5e-5, f"bidirectional lstm+snake D={D}")
    with pytest.raises(NotImplementedError):
        m.run(x.to(dev), return_state=True)
    assert L.load().bc_lstm_status(1) == 0


@pytest.mark.parametrize("Cin,Cout,K,d,T,cfg", [
    (192, 192, 7, 3, 1200, 322), (384, 384, 7, 9, 700, 322), (192, 192, 7, 1, 2000, 222), (192, 192, 7, 3, 1200, 122),
    (384, 384, 1, 1, 1000, 314), (192, 192, 1, 1, 1000, 322), (768, 768, 1, 1, 520, 214), (384, 384, 1, 1, 1000, 114),
    (384, 384, 1, 1, 1000, 122)])
def test_b4_staging_bit_identical_to_single_float(dev, Cin, Cout, K, d, T, cfg):
    """16-byte input staging (B4: stride-1 launches whose rows are 16-byte aligned with Tin % 4 == 0) stages the
    same values, block maxima and LDS image as the single-float staging, which runs when the input is not 16-byte
    aligned: an aligned and a 4-byte-offset copy of the same input give bit-identical outputs (k7 16-wave tiles,
    pointwise 192 x 128 and 16-wave tiles; h3, bf16, x6), within the conv tolerance of the oracle in h3 / x6."""
    prec = {1: "x6", 2: "bf16", 3: "h3"}[cfg // 100]
    old = L.precision_mode()
    L.set_precision(prec)
    try:
        g = torch.Generator().manual_seed(Cin + Cout * 3 + K + d)
        pad = K // 2 * d
        m = CV.WNConv1d(Cin, Cout, kernel_size=K, dilation=d, padding=pad)
        conv = _rand_wn_conv(m, g)
        B = 2
        x = torch.randn(B, Cin, T, generator=g)
        res = torch.randn(B, Cout, T, generator=g)
        sd = {k: v.detach() for k, v in conv.state_dict().items()}
        want = O.conv(x, sd, "", K, 1, pad, d, False) + res
        m.to(dev)
        st = torch.cuda.current_stream().cuda_stream
        wp, bias = m.packed_as(cfg, dev)
        buf = torch.empty(B * Cin * T + 4, device=dev)
        outs = []
        for off in (0, 1):  # the allocation is 256-B aligned: offset 0 takes B4, offset 1 float the single-float path
            xd = buf[off:off + B * Cin * T].view(B, Cin, T)
            xd.copy_(x.to(dev))
            rd = res.to(dev)
            y = torch.empty(B, Cout, T, device=dev)
            L.call("bc_conv1d_fwd", xd.data_ptr(), wp.data_ptr(), L.ptr(bias), rd.data_ptr(), 0, 0, y.data_ptr(), 0,
                   B, Cin, T, Cout, T, K, 1, d, pad, 0, cfg, st)
            torch.cuda.synchronize()
            outs.append(y.cpu())
        assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max()
        tol = 3e-6 * max(1.0, np.sqrt(Cin * K / 64)) if prec != "bf16" else 2e-2
        assert_close_rel(outs[0], want, tol, f"{prec} cfg {cfg}")
    finally:
        L._mode = old


@pytest.mark.parametrize("Cin,Cout,K,d,B,T", [(768, 768, 7, 1, 16, 25), (384, 384, 7, 3, 4, 125), (1024, 1536, 7, 1, 3, 5),
                                             (192, 192, 7, 9, 2, 60), (1536, 1536, 7, 1, 64, 24), (768, 768, 7, 9, 64, 120),
                                             (768, 768, 1, 1, 16, 25), (384, 384, 1, 1, 16, 125), (1536, 1536, 1, 1, 64, 24),
                                             (1536, 1024, 3, 1, 16, 6)])
@pytest.mark.parametrize("prec", ["x6", "bf16", "h3"])
def test_narrow_launch_tile(dev, Cin, Cout, K, d, B, T, prec):
    """bc_conv1d_select_cfg_n (ABI 15): a stride-1 k7 conv with <= 128 output columns per clip (a streaming chunk, a
    small batch) leaves the 16-wave 192 x 256 tile for a narrower one, a pointwise conv the 192 x 128 tile for a
    64-column one; the module picks it by itself.  The same K
    order per output makes x6 and bf16 results bit-identical on either tile; h3 (block scales per staged tile) agrees
    to fp32 rounding and matches the fp64 oracle at the conv tolerance."""
    old = L.precision_mode()
    L.set_precision(prec)
    try:
        g = torch.Generator().manual_seed(Cin + 7 * d + T + K)
        pad = (K - 1) // 2 * d
        m = CV.WNConv1d(Cin, Cout, kernel_size=K, dilation=d, padding=pad)
        conv = _rand_wn_conv(m, g)
        x = torch.randn(B, Cin, T, generator=g)
        sd = {k: v.detach() for k, v in conv.state_dict().items()}
        m.to(dev)
        xd = x.to(dev)
        lib = L.load()
        wide = lib.bc_conv1d_select_cfg(Cout, Cin, K, 1, d, L.precision_mode())
        narrow = lib.bc_conv1d_select_cfg_n(Cout, Cin, K, 1, d, L.precision_mode(), B, T)
        # (x6 multi-tap convs: the register-A tile 120, conv1d_x6ra.hip)
        assert wide % 100 in ((22, 21, 20) if K > 1 else (14, 22)) and narrow != wide, (wide, narrow)
        st = torch.cuda.current_stream().cuda_stream
        outs = {}
        for cfg in (wide, narrow):
            wp, bias = m.packed_as(cfg, dev)
            y = torch.empty(B, Cout, T, device=dev)
            L.call("bc_conv1d_fwd", xd.data_ptr(), wp.data_ptr(), L.ptr(bias), 0, 0, 0, y.data_ptr(), 0,
                   B, Cin, T, Cout, T, K, 1, d, pad, 0, cfg, st)
            outs[cfg] = y
        via_module = m(xd)
        torch.cuda.synchronize()
    finally:
        L._mode = old
    a, b = outs[wide].cpu(), outs[narrow].cpu()
    assert torch.equal(via_module.cpu(), b), "the module runs the narrow tile"
    if prec in ("x6", "bf16"):
        assert torch.equal(a, b), (a - b).abs().max()
    else:
        assert_close_rel(b, a, 2e-6, "h3 narrow vs 16-wave tile")
    if prec == "h3":
        want = O.conv(x, sd, "", K, 1, pad, d, False)
        assert_close_rel(b, want, 3e-6 * max(1.0, np.sqrt(Cin * K / 64)), "h3 narrow tile vs oracle")


@pytest.mark.parametrize("d", [1, 9])
def test_strip_partition_independent(dev, d):
    """The C = 48 strip kernel sizes its strips by the launch (8 blocks of 128 columns, fewer when B * blocks / 8
    would leave CUs without a strip): 64 clips of 1254 samples run strips of 2 blocks, their first 16 (or 1) alone
    strips of 1 block; 4 clips of 24 000 samples strips of 2, one of them alone strips of 1.  The per-block arithmetic (block scales, the carried or
    reloaded halo) does not depend on the partition: the shared clips come out bit-identical."""
    old = L.precision_mode()
    L.set_precision("h3")
    try:
        g = torch.Generator().manual_seed(4800 + d)
        ru = BL.ResidualUnit(48, dilation=d)
        _rand_wn_conv(ru.block[1], g)
        _rand_wn_conv(ru.block[3], g)
        for k in (0, 2):
            ru.block[k].act.load_state_dict(_snake(48, g).state_dict())
        ru.to(dev)
        assert L.resunit_kernel_name(ru._fused_cfg(), 48, d).startswith("resunit_strip_kernel")
        x = torch.randn(64, 48, 1254, generator=g).to(dev)
        y64 = ru(x)
        y16 = ru(x[:16].contiguous())
        y1 = ru(x[:1].contiguous())
        long = torch.randn(4, 48, 24000, generator=g).to(dev)
        yl = ru(long)
        yl1 = ru(long[1:2].contiguous())
        torch.cuda.synchronize()
    finally:
        L._mode = old
    assert torch.equal(y16, y64[:16]) and torch.equal(y1, y64[:1])
    assert torch.equal(yl1, yl[1:2])


def test_launch_timer_records_the_composite_calls(dev):
    """bc_launch_timer_* (ABI 17): with the timer on, a ResLSTM forward records its transposes, input projection and
    persistent recurrence (the variant name lstm_seq_launch ran, as rocprofv3 spells it), and a VQ forward its kernel,
    each with an event time and the launch's algorithmic work; KernelTimer merges them; nothing is recorded when off."""
    old = L.precision_mode()
    L.set_precision("x6")
    try:
        H, B, T = 1536, 64, 40
        g = torch.Generator().manual_seed(7)
        m = BL.ResLSTM(H, num_layers=2).to(dev)
        x = torch.randn(B, H, T, generator=g).to(dev)
        m(x)  # packing and warm-up outside the timer
        torch.cuda.synchronize()
        tm = L.KernelTimer()
        L.set_timer(tm)
        m(x)
        L.set_timer(None)
        summ = tm.summary()
        m(x)  # timer off: nothing more is recorded
        torch.cuda.synchronize()
        tm.drain_library()
    finally:
        L._mode = old
    names = set(summ)
    rec = [k for k in names if k.startswith("lstm_seq2_x6_kernel<12, 3, ")]
    assert rec and summ[rec[0]]["launches"] == 2, names
    assert summ[rec[0]]["flops_total"] == 2 * 2.0 * 4 * H * H * T * B
    assert summ["btc_to_ctb_kernel"]["launches"] == 1 and summ["ctb_to_btc_add_kernel"]["launches"] == 1
    proj = [k for k in names if k.startswith(("pw_presplit_x6_kernel", "conv1d_x6_kernel"))]
    assert proj and sum(summ[k]["launches"] for k in proj) == 2, names
    assert all(d["ms_total"] > 0 for d in summ.values())
    assert len(tm.lib_records) == sum(d["launches"] for d in summ.values())  # the off-period added nothing
