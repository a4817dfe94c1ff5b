"""resunit_rr at C = 48 against the CPU oracle over dilations 1-9, clip lengths and batch sizes (the probe that
found the 16x16x16-onto-16x16x32 accumulator hazard; prints the bad columns / channels of a failing case)."""
import sys, torch
import os
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
from audiotokenization_amd import _lib as L, blocks as BL, modules as M
from oracle import bigcodec_oracle as O
from test_gpu_kernels import _rand_wn_conv, _snake
L.set_precision("h3")
dev = torch.device("cuda", 0)
for (C, d, B, T) in [(48, 3, 1, 1001), (48, 3, 1, 4096), (48, 1, 1, 24000), (48, 9, 1, 24000), (48, 3, 2, 700), (48, 2, 1, 1001), (48, 4, 1, 1001), (48, 5, 1, 1001)]:
    g = torch.Generator().manual_seed(C * 10 + d)
    ru = BL.ResidualUnit(C, dilation=d)
    _rand_wn_conv(ru.block[1], g); _rand_wn_conv(ru.block[3], g)
    for k in (0, 2):
        s = _snake(C, g); ru.block[k].act.load_state_dict(s.state_dict())
    x = torch.randn(B, C, T, generator=g)
    sd = {k: v.detach() for k, v in ru.state_dict().items()}
    want = O.residual_unit(x, sd, "", d, False, False)
    ru.to(dev)
    got = ru.flow(x.to(dev), None)[0].cpu()
    err = ((got - want).abs().max() / want.abs().max()).item()
    bad = ((got - want).abs() > 1e-3 * want.abs().max())
    cols = torch.nonzero(bad.any(1).any(0)).flatten()
    chans = torch.nonzero(bad.any(2).any(0)).flatten()
    print(f"C={C} d={d} B={B} T={T}: err {err:.2e}, bad cols {cols[:10].tolist()} (n={cols.numel()}), bad chans {chans[:20].tolist()}", flush=True)
