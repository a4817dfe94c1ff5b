"""torch.ops.bigcodec.* on the MI355X: torch.library.opcheck (schema / fake-tensor / aot-dispatch
consistency of csrc/torch_ops.cpp with the fake kernels in audiotokenization_amd/ops.py) on the
arguments the codec modules pass, and the ops equal the raw C ABI called through ctypes."""
import pytest
import torch

from helpers import build_models

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def base(dev):
    return build_models("base", device=dev)


def _cases(dev, base):
    from audiotokenization_amd import _lib as L
    from audiotokenization_amd import synth
    from audiotokenization_amd.blocks import EncoderBlock, ResidualUnit, ResLSTM

    enc, dec, *_ = base
    g = torch.Generator().manual_seed(7)
    x1 = torch.from_numpy(synth.synth_clips(2, 4000, clip0=1)).unsqueeze(1).to(dev)
    cases = []
    first = enc.block[0]
    wp, bias, cfg = first.prepared(dev)
    cases.append(("conv1d", (x1, wp, bias, None, None, None, first.out_channels, 4000, 7, 1, 1, 3, 0, cfg, False)))
    blk = next(m for m in enc.block if isinstance(m, EncoderBlock))
    ru = blk.block[0]
    assert isinstance(ru, ResidualUnit)
    C = ru.block[1].in_channels
    x = torch.randn(2, C, 300, generator=g).to(dev)
    a, ib = ru.block[0].act.coeffs(dev)
    cases.append(("snake", (x, a, ib)))
    cases.append(("tanh", (x,)))
    cfg = ru._fused_cfg()
    if cfg >= 0:
        from audiotokenization_amd.blocks import _conv_of
        c7, c1 = _conv_of(ru.block[1]), _conv_of(ru.block[3])
        w7, b7 = c7.packed_as(cfg, dev)
        w1, b1 = c1.packed_as(cfg, dev)
        ma, mb = ru.block[2].act.coeffs(dev)
        cases.append(("resunit", (x, None, a, ib, w7, b7, ma, mb, w1, b1, None, None, c7.dilation, c7.pad_left(), cfg,
                                  False)))
    lstm = next(m for m in enc.block if isinstance(m, ResLSTM))
    H = lstm.lstm.hidden_size
    (wih, whh, lb), _ = lstm.lstm.prepared(dev)
    xl = torch.randn(2, H, 9, generator=g).to(dev)
    cases.append(("reslstm", (xl, wih, lb, whh, None, None, L.precision_mode(), None, None, True)))
    from audiotokenization_amd import modules as M

    act = M.Activation1d(M.SnakeBeta(C, alpha_logscale=True), antialias=True, up_ratio=3, down_ratio=2).to(dev)
    fu, fd = act.filters(dev)
    cases.append(("aa_snake_ex", (x, a, ib, fu, fd, 3, 2)))
    bl = ResLSTM(64, num_layers=1, bidirectional=True).to(dev)
    (bwih, bwhh, bb), _ = bl.lstm.prepared(dev)
    cases.append(("reslstm_bidir", (torch.randn(2, 64, 7, generator=g).to(dev), bwih, bb, bwhh, None, None,
                                    L.precision_mode())))
    fvq = dec.quantizer.layers[0]
    cb, cbn, csq, w_in, b_in, w_out, b_out = fvq.prepared(dev)
    z = torch.randn(2, fvq.dim, 11, generator=g).to(dev)
    cases.append(("vq", (z, w_in, b_in, cb, cbn, csq, w_out, b_out, True, True)))
    cases.append(("vq_prepare_codebook", (cb,)))
    idx = torch.randint(0, 8192, (2, 11, 1), generator=g).to(dev)
    cases.append(("vq2emb", (idx, 0, cb, w_out, b_out)))
    cst, wst, bst = dec.quantizer.prepared_stack(dev)
    cases.append(("vq2emb_ct", (idx, cst, wst, bst)))
    fq = M.FSQ([4, 4, 4, 8], dim=64, channel_first=True).eval()
    fw_in, fb_in, fw_out, fb_out, fconsts = fq.prepared(dev)
    cases.append(("fsq", (torch.randn(2, 64, 13, generator=g).to(dev), fw_in, fb_in, fw_out, fb_out, fconsts)))
    cases.append(("fsq_codes", (torch.randint(-600, 1200, (2, 13), generator=g).to(dev), fw_out, fb_out, fq.levels)))
    return cases


def test_opcheck_every_codec_op(dev, base):
    from audiotokenization_amd import ops

    ns = ops.load()
    seen = set()
    for name, args in _cases(dev, base):
        torch.library.opcheck(getattr(ns, name).default, args)
        seen.add(name)
    assert {"conv1d", "snake", "tanh", "reslstm", "reslstm_bidir", "vq", "vq2emb", "vq2emb_ct", "fsq", "fsq_codes"} <= seen


def test_ops_equal_the_raw_c_abi(dev, base):
    """The dispatcher path computes exactly what the ctypes call of the same entry point computes."""
    from audiotokenization_amd import _lib as L
    from audiotokenization_amd import ops

    ns = ops.load()
    enc, *_ = base
    first = enc.block[0]
    wp, bias, cfg = first.prepared(dev)
    from audiotokenization_amd import synth

    x = torch.from_numpy(synth.synth_clips(3, 5000, clip0=4)).unsqueeze(1).to(dev)
    y_op = ns.conv1d(x, wp, bias, None, None, None, first.out_channels, 5000, 7, 1, 1, 3, 0, cfg, False)[0]
    y_c = torch.empty_like(y_op)
    L.call("bc_conv1d_fwd", x.data_ptr(), wp.data_ptr(), L.ptr(bias), None, None, None, y_c.data_ptr(), None, 3, 1,
           5000, first.out_channels, 5000, 7, 1, 1, 3, 0, cfg, L.stream_of(x))
    xs = torch.empty(2, 1, 777, device=dev)
    ns.synth_clips_(xs, 9)
    xs_c = torch.empty_like(xs)
    L.call("bc_synth_clips", xs_c.data_ptr(), 2, 777, 9, L.stream_of(xs_c))
    torch.cuda.synchronize()
    assert torch.equal(y_op, y_c) and torch.equal(xs, xs_c)


def test_ops_reject_bad_inputs_loudly(dev):
    from audiotokenization_amd import ops

    ns = ops.load()
    with pytest.raises((RuntimeError, NotImplementedError)):  # no CPU kernel is registered: no silent fallback
        ns.snake(torch.zeros(1, 2, 3), torch.zeros(2), torch.zeros(2))
    x = torch.zeros(1, 2, 3, device=dev)
    with pytest.raises(ValueError, match="coefficients"):
        ns.snake(x, torch.zeros(3, device=dev), torch.zeros(3, device=dev))
    with pytest.raises(RuntimeError, match="contiguous"):
        ns.tanh(torch.zeros(4, 3, device=dev).t())
