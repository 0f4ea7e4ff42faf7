"""LDS-DMA convolution (conv_glds_x3) on split-layout inputs (s2v_split_act), MI355X only.

The kernel stages both operands global -> LDS with global_load_lds; its K-slice order, MFMA
fragments and product order are the register-staged x3 kernel's, so on the same input and the same
split-K factor the two give the same bits.  Also checked against an fp64 torch reference with the
split precision's bound, and the split layout itself byte by byte.
"""
import math

import pytest
import torch
import torch.nn.functional as F

import s2v_import  # noqa: F401

pytestmark = pytest.mark.gpu

from s2v_amd import ops  # noqa: E402
from s2v_amd.ops import NHWC, ConvW  # noqa: E402

DEV = "cuda"
REL = {"bf16x3": 5e-5, "f16x3": 3e-6}


@pytest.fixture(scope="module")
def ctx():
    return ops.Ctx(DEV)


@pytest.fixture(params=["bf16x3", "f16x3"])
def sprec(request):
    prev = ops.set_precision(request.param)
    yield request.param
    ops.set_precision(prev)


def rnd(*shape, seed=0, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return lo + (hi - lo) * torch.rand(*shape, generator=g, dtype=torch.float64)


def nhwc(t):
    return NHWC(t.permute(0, 2, 3, 1).contiguous().to(DEV))


@pytest.mark.parametrize("c,cs", [(32, 32), (96, 128)])
def test_split_act_layout(ctx, sprec, c, cs):
    """[hi 32 | lo 32] 16-bit per pixel and 32-channel block, hi = T(v), lo = T(v - hi), RNE."""
    x = rnd(2, 5, 7, cs, seed=1) * 3
    xv = NHWC(x.float().to(DEV)).slice(0, c)
    out = NHWC.empty(2, 5, 7, c, DEV)
    ops.split_act(ctx, xv, out)
    raw = out.t.view(torch.int16).reshape(2, 5, 7, c // 32, 2, 32).cpu()
    dt = torch.float16 if sprec == "f16x3" else torch.bfloat16
    hi, lo = raw[..., 0, :].view(dt).float(), raw[..., 1, :].view(dt).float()
    v = x[..., :c].float().reshape(2, 5, 7, c // 32, 32)
    assert torch.equal(hi, v.to(dt).float())
    assert torch.equal(lo, (v - hi).to(dt).float())


GLDS_CASES = [
    # (n, cin, h, w, cout, k, stride, pad, splits (0: 1), pool, modulated)
    (2, 64, 17, 19, 96, 3, 1, 1, 0, False, False),       # 256x128 tile, ragged M
    (2, 64, 16, 16, 256, 3, 1, 1, 0, False, False),      # 256x256 tile
    (1, 96, 9, 11, 320, 3, 1, 1, 2, False, False),       # N tail past 256, split-K
    (2, 32, 20, 12, 64, 3, 2, 1, 0, False, False),       # stride 2
    (2, 128, 12, 12, 128, 2, 2, 0, 0, False, False),     # ResBlock skip as a 2x2 stride-2 conv
    (2, 64, 14, 10, 40, 1, 1, 0, 3, False, False),       # 1x1, split-K
    (2, 64, 16, 12, 128, 3, 1, 1, 1, True, False),       # pooled epilogue (ResBlock conv1)
    (3, 64, 10, 12, 96, 3, 1, 1, 0, False, True),        # per-sample modulated weights
    (2, 32, 40, 40, 32, 5, 1, 2, 0, False, False),       # 25 taps
]


@pytest.mark.parametrize("case", GLDS_CASES, ids=[str(i) for i in range(len(GLDS_CASES))])
def test_glds_conv_matches_x3_kernel(ctx, sprec, case):
    n, cin, h, w, cout, k, stride, pad, splits, pool, modulated = case
    splits = splits or 1          # the two planners pick their own K splits: pin one for the bitwise check
    wt = rnd(cout, cin, k, k, seed=11) / math.sqrt(cin * k * k)
    bias = rnd(cout, seed=12)
    x = rnd(n, cin, h, w, seed=13)
    res = None
    cw = ConvW(wt.float(), bias.float(), DEV, stride=stride, padding=pad)
    oh, ow = cw.out_hw(h, w)
    f = 2 if pool else 1
    xv = nhwc(x.float())
    xs = ops.split_act(ctx, xv)
    outs = []
    for inp in (xv, xs):
        y = NHWC.empty(n, oh // f, ow // f, cout, DEV)
        if modulated:
            s = rnd(n, cin, seed=14, lo=0.5, hi=1.5).float().to(DEV)
            d = rnd(n, cout, seed=15, lo=0.5, hi=1.5).float().to(DEV)
            ops.modulated_conv2d(ctx, inp, cw, y, s, d, act=ops.ACT_LRELU, alpha=0.2, force_splits=splits)
        else:
            if not pool:
                res = nhwc(rnd(n, cout, oh, ow, seed=16).float())
            ops.conv2d(ctx, inp, cw, y, act=ops.ACT_LRELU, alpha=0.2, res=res, pool=pool, force_splits=splits)
        outs.append(y.t.cpu())
    assert torch.equal(outs[0], outs[1]), f"max diff {(outs[0] - outs[1]).abs().max():.3e}"
    if not modulated:
        ref = F.conv2d(x, wt, bias, stride, pad)
        if res is not None:
            ref = ref + res.t.permute(0, 3, 1, 2).double().cpu()
        ref = F.leaky_relu(ref, 0.2)
        bound = F.conv2d(x.abs(), wt.abs(), None, stride, pad) + 2
        if pool:
            ref, bound = F.avg_pool2d(ref, 2), F.avg_pool2d(bound, 2)
        got = outs[1].permute(0, 3, 1, 2).double()
        assert ((got - ref).abs() <= REL[sprec] * bound + 1e-6).all()


def test_glds_plan_reports_the_kernel(ctx, sprec):
    x = NHWC.empty(2, 16, 16, 64, DEV)
    xs = ops.split_act(ctx, x)
    for cout, bn in ((96, 128), (256, 256)):
        cw = ConvW(torch.randn(cout, 64, 3, 3), None, DEV, padding=1)
        y = NHWC.empty(2, 16, 16, cout, DEV)
        captured = {}
        ops.CONV_HOOK = lambda c, p, fl, launch: captured.setdefault("p", p)
        try:
            ops.conv2d(ctx, xs, cw, y)
        finally:
            ops.CONV_HOOK = None
        sym = ops.conv_symbol(ctx, captured["p"])
        assert sym.startswith(f"void s2v::conv_glds_x3<256, {bn},"), sym


def test_split_input_rejected_where_unsupported(ctx, sprec):
    """A split-layout input only feeds the LDS-DMA kernel: reflect padding / prologues raise."""
    x = NHWC.empty(1, 8, 8, 32, DEV)
    xs = ops.split_act(ctx, x)
    y = NHWC.empty(1, 8, 8, 32, DEV)
    cw = ConvW(torch.randn(32, 32, 3, 3), None, DEV, padding=1, pad_mode=ops.PAD_REFLECT)
    with pytest.raises(Exception):
        ops.conv2d(ctx, xs, cw, y)
    cw = ConvW(torch.randn(32, 32, 3, 3), None, DEV, padding=1)
    with pytest.raises(Exception):
        ops.conv2d(ctx, xs, cw, y, pre_act=ops.ACT_LRELU, pre_alpha=0.2)


@pytest.mark.parametrize("case", [GLDS_CASES[0], GLDS_CASES[5], GLDS_CASES[6], GLDS_CASES[7]],
                         ids=["ragged", "1x1-splitk", "pooled", "modulated"])
def test_glds_512x128_tile(ctx, sprec, case):
    """The 512x128 configuration (the planner's pick for N <= 128 on large M), forced on the small
    cases through the planner knob."""
    prev = ops.tune(ctx, ops.TUNE_GLDS_TILE, 2)
    try:
        test_glds_conv_matches_x3_kernel(ctx, sprec, case)
    finally:
        ops.tune(ctx, ops.TUNE_GLDS_TILE, prev)


def test_split_input_of_another_precision_raises(ctx, sprec):
    """A tensor split in one precision is not read as the other's halves (bf16 vs f16 layout)."""
    x = NHWC.empty(1, 8, 8, 32, DEV)
    xs = ops.split_act(ctx, x)
    other = "f16x3" if sprec == "bf16x3" else "bf16x3"
    y = NHWC.empty(1, 8, 8, 32, DEV)
    cw = ConvW(torch.randn(32, 32, 3, 3), None, DEV, padding=1)
    prev = ops.set_precision(other)
    try:
        with pytest.raises(ops._lib.S2VError, match="split layout"):
            ops.conv2d(ctx, xs, cw, y)
        ops.set_precision("f32")
        with pytest.raises(ops._lib.S2VError, match="split layout"):
            ops.conv2d(ctx, xs, cw, y)
    finally:
        ops.set_precision(prev)
