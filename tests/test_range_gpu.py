"""f16x3 activation range guard (ops.RANGE_GUARD).

f16 halves cover |v| < 65504 and a lo half turns subnormal below 2^-3: a layer whose input leaves
that range gets a calibrated power-of-two pre-scale (s2v_conv_params.x_scale), and an input that
still overflows later sets the lane's non-finite flag (check_range raises)."""
import math

import pytest
import torch
import torch.nn.functional as F

import s2v_import  # noqa: F401
from s2v_amd import _lib, ops
from s2v_amd.ops import NHWC, ConvW

pytestmark = pytest.mark.gpu
DEV = "cuda"
REL = 3e-6          # f16x3 per-product bound (as tests/test_conv_glds_gpu.py), relative to |x| * |w|


@pytest.fixture
def f16x3():
    prev = ops.set_precision("f16x3")
    yield
    ops.set_precision(prev)


def _case(seed, cin=64, cout=96, h=13, w=11):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(2, cin, h, w, generator=g, dtype=torch.float64) * 2 - 1
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) / math.sqrt(cin * 9)
    return x, wt


@pytest.mark.parametrize("mag", [6e4, 1e5, 1e-6, 3.0])
def test_conv_inputs_outside_the_f16_range(f16x3, mag):
    x, wt = _case(1)
    x = x * mag
    ctx = ops.Ctx(DEV)
    cw = ConvW(wt.float(), None, DEV, padding=1)
    xv = NHWC(x.permute(0, 2, 3, 1).float().contiguous().to(DEV))
    y = NHWC.empty(2, 13, 11, 96, DEV)
    ops.conv2d(ctx, xv, cw, y)
    ctx.check_range()                                    # no overflow with the calibrated pre-scale
    got = y.t.permute(0, 3, 1, 2).double().cpu()
    ref = F.conv2d(x.float().double(), wt.float().double(), None, 1, 1)
    bound = F.conv2d(x.float().double().abs(), wt.float().double().abs(), None, 1, 1)
    assert torch.isfinite(got).all()
    assert ((got - ref).abs() <= REL * bound + 1e-30).all(), float(((got - ref).abs() / (bound + 1e-30)).max())
    expect = ops.x_scale_for(float(x.float().abs().max()))
    assert cw._xscale[ops.PREC_F16X3] == expect and (expect != 1.0) == (mag != 3.0)


def test_overflow_after_calibration_is_flagged(f16x3):
    x, wt = _case(2)
    ctx = ops.Ctx(DEV)
    cw = ConvW(wt.float(), None, DEV, padding=1)
    y = NHWC.empty(2, 13, 11, 96, DEV)
    small = NHWC((x * 10).permute(0, 2, 3, 1).float().contiguous().to(DEV))
    ops.conv2d(ctx, small, cw, y)                        # calibrates: no pre-scale needed
    ctx.check_range()
    big = NHWC((x * 1e6).permute(0, 2, 3, 1).float().contiguous().to(DEV))
    ops.conv2d(ctx, big, cw, y)                          # far outside the calibrated range
    with pytest.raises(_lib.S2VError, match="non-finite"):
        ctx.check_range()
    ctx.check_range()                                    # the flag was reset


def test_modulated_conv_range(f16x3):
    x, wt = _case(3, cin=32, cout=64)
    x = x * 2e5
    ctx = ops.Ctx(DEV)
    cw = ConvW(wt.float(), None, DEV, padding=1)
    xv = NHWC(x.permute(0, 2, 3, 1).float().contiguous().to(DEV))
    y = NHWC.empty(2, 13, 11, 64, DEV)
    s = torch.full((2, 32), 0.5, device=DEV)
    d = torch.full((2, 64), 2.0, device=DEV)
    ops.modulated_conv2d(ctx, xv, cw, y, s, d)
    ctx.check_range()
    got = y.t.permute(0, 3, 1, 2).double().cpu()
    ref = F.conv2d(x.float().double(), wt.float().double(), None, 1, 1)      # 0.5 * 2.0 = 1
    bound = F.conv2d(x.float().double().abs(), wt.float().double().abs(), None, 1, 1)
    assert torch.isfinite(got).all() and ((got - ref).abs() <= 2 * REL * bound).all()


def test_in_scale_operand_is_what_calibrates(f16x3):
    """A StyleGAN2 modulated input (in_scale, GPEN / GFPGAN) is split as x * in_scale: the calibration
    measures that operand (max |x| * max |in_scale|), so an in_scale that lifts an in-range x past the
    f16 ceiling still gets a pre-scale and the result stays finite and within the f16x3 bound."""
    x, wt = _case(4)
    ctx = ops.Ctx(DEV)
    cw = ConvW(wt.float(), None, DEV, padding=1)
    xv = NHWC(x.permute(0, 2, 3, 1).float().contiguous().to(DEV))
    y = NHWC.empty(2, 13, 11, 96, DEV)
    s = torch.full((2, 64), 2.0e5, device=DEV)
    ops.conv2d(ctx, xv, cw, y, in_scale=s)
    ctx.check_range()
    assert cw._xscale[ops.PREC_F16X3] < 1.0
    xs = x.float().double() * 2.0e5
    got = y.t.permute(0, 3, 1, 2).double().cpu()
    ref = F.conv2d(xs, wt.float().double(), None, 1, 1)
    bound = F.conv2d(xs.abs(), wt.float().double().abs(), None, 1, 1)
    assert torch.isfinite(got).all() and ((got - ref).abs() <= REL * bound + 1e-30).all()


def test_in_scale_overflow_after_calibration_is_flagged(f16x3):
    """Calibrated with in_scale 1, then an in_scale of 1e6 pushes the split operand over 65504: the
    launch flags it and check_range raises (never silent)."""
    x, wt = _case(5)
    ctx = ops.Ctx(DEV)
    cw = ConvW(wt.float(), None, DEV, padding=1)
    xv = NHWC((x * 100).permute(0, 2, 3, 1).float().contiguous().to(DEV))
    y = NHWC.empty(2, 13, 11, 96, DEV)
    ops.conv2d(ctx, xv, cw, y, in_scale=torch.ones((2, 64), device=DEV))
    ctx.check_range()
    ops.conv2d(ctx, xv, cw, y, in_scale=torch.full((2, 64), 1.0e6, device=DEV))
    with pytest.raises(_lib.S2VError, match="non-finite"):
        ctx.check_range()


def test_scale_up_keeps_headroom():
    """A small-range layer is scaled into [2^9, 2^10): 64x headroom below the f16 ceiling for later
    batches, and in-range layers keep x_scale 1."""
    for amax in (1e-6, 0.01, 0.1):
        m = amax * ops.x_scale_for(amax)
        assert 2 ** 9 <= m < 2 ** 10
    assert ops.x_scale_for(0.5) == 1.0 and ops.x_scale_for(1e4) == 1.0
    assert 2 ** 9 <= 1e5 * ops.x_scale_for(1e5) < 2 ** 10


def test_model_forward_out_of_range_batch_reruns_in_bf16x3(f16x3):
    """An eager model forward whose batch leaves the range calibrated on the first forward (face
    input 1e5 x larger: the first conv's split operand passes 65504) reads the lane's flag when it
    returns and runs again in bf16x3: the returned output is the bf16x3 forward's, bit for bit, not
    inf / NaN; in-range forwards return f16x3 outputs without a re-run."""
    from helpers import synth_sd
    from s2v_amd import models
    net = models.LNet()
    net.load_state_dict(synth_sd("lnet"), strict=True)
    net.eval()
    g = torch.Generator(device=DEV).manual_seed(7)
    mel = torch.rand((2, 1, 80, 16), generator=g, device=DEV) * 8 - 4
    face = torch.rand((2, 6, 96, 96), generator=g, device=DEV)
    net(mel, face)                                       # first forward: calibration
    ctx = net._s2v_engines[str(face.device)][1][0]
    assert ctx.reruns == 0
    ok = net(mel, face)
    assert ctx.reruns == 0 and torch.isfinite(ok).all()
    big = face * 1.0e5
    out = net(mel, big)
    assert ctx.reruns == 1 and torch.isfinite(out).all()
    with ops.precision("bf16x3"):
        ref = net(mel, big)
    assert torch.equal(out, ref)


def test_first_forward_out_of_range_recalibrates(f16x3):
    """the engine's first (calibration) forward at a face input 1e5 x larger.  The first conv's
    split operand passes 65504, so in the unscaled calibration pass every layer behind it measures a
    non-finite amax.  Those layers stay uncalibrated and the next pass calibrates them again behind the
    now pre-scaled first conv (ops.end_forward -> "recalibrate"): no layer keeps a scale measured from
    inf / NaN, nothing falls back to bf16x3, and the output matches the exact-f32 forward."""
    from helpers import synth_sd
    from s2v_amd import models
    net = models.LNet()
    net.load_state_dict(synth_sd("lnet"), strict=True)
    net.eval()
    g = torch.Generator(device=DEV).manual_seed(11)
    mel = torch.rand((2, 1, 80, 16), generator=g, device=DEV) * 8 - 4
    big = torch.rand((2, 6, 96, 96), generator=g, device=DEV) * 1.0e5
    out = net(mel, big)                                  # first forward: calibration passes
    eng, lanes = net._s2v_engines[str(big.device)]
    ctx = lanes[0]
    assert ctx.reruns == 0 and torch.isfinite(out).all()
    amaxes = []

    def walk(o, seen):
        if id(o) in seen:
            return
        seen.add(id(o))
        if isinstance(o, ConvW) and ops.PREC_F16X3 in o.__dict__.get("_xscale", {}):
            amaxes.append(o.x_amax)            # (a ConvW's launched forms: .rowpack / .poly, walked below)
        if isinstance(o, (list, tuple)):
            for v in o:
                walk(v, seen)
        elif isinstance(o, dict):
            for v in o.values():
                walk(v, seen)
        elif hasattr(o, "__dict__") and type(o).__module__.startswith("s2v_amd"):
            for v in vars(o).values():
                walk(v, seen)
    walk(eng, set())
    assert len(amaxes) > 100 and all(math.isfinite(m) for m in amaxes)
    assert max(amaxes) > 65504                           # the first conv's operand, scaled down
    with ops.precision("f32"):
        ref = net(mel, big)
    d = (out - ref).abs()
    assert float(d.max()) <= 1e-4 and float(d.mean()) <= 1e-5, (float(d.max()), float(d.mean()))
