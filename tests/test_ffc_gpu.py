"""LNet's fused FFC kernels (csrc/ffc.hip: ffc_spec_fwd / ffc_spec_inv / ffc_norm) against the separate
launches they replace (st1 conv -> rfft2 -> fu conv -> irfft2 -> st2 conv -> InstanceNorm/ADAIN; the engine's
S2V_LNET_FUSED path), one
FineADAINLama of each decoder level (models/base_blocks.py:368-386, models/ffc.py:60-233), in both
split-precision arithmetics, with the reflect-padded output and the FFCResnetBlock residual, at B = 2 and
at the benchmarked B = 16 (the XCD-grouped block order); and a whole fused-path LNet forward against the
reference golden."""
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import synth_sd
from s2v_amd import ops
from s2v_amd.ops import NHWC

pytestmark = pytest.mark.gpu
DEV = "cuda"
# fused vs separate launches: the same split-precision products in another summation order, then the
# InstanceNorm (unit variance outputs): max |diff| bounds per arithmetic
TOL = {"f16x3": 5e-5, "bf16x3": 2e-3}


def _engine():
    from s2v_amd.engine import lnet
    return lnet, lnet.LNetEngine(synth_sd("lnet"), torch.device(DEV))


@pytest.mark.parametrize("prec", ["f16x3", "bf16x3"])
@pytest.mark.parametrize("level", [0, 1, 2])
@pytest.mark.parametrize("b", [2, 16])
def test_ffc_fused_matches_separate(monkeypatch, prec, level, b):
    lnet, eng = _engine()
    monkeypatch.setattr(lnet, "FUSED_LEVELS", (12, 24, 48))
    lv = eng.levels[level]
    f1, f2 = lv["blocks"][3]
    h, c = f1.h, f1.c
    g = torch.Generator(device=DEV).manual_seed(100 + level)
    x = NHWC(torch.randn(b, h, h, c, generator=g, device=DEV))
    xpad = NHWC.empty(b, h + 2, h + 2, c, DEV)
    ctx = ops.Ctx(DEV)
    ops.pad_reflect(ctx, x, xpad, (1, 1, 1, 1))
    # ADAIN parameters from the real heads on a random audio feature
    z = NHWC(torch.randn(b, 1, 1, eng.bank.layer1.cin, generator=g, device=DEV))
    prev = ops.set_precision(prec)
    try:
        params = eng.bank.run(ctx, z)
        outs = {}
        for fused in (False, True):
            monkeypatch.setattr(lnet, "FUSED", fused)
            y = NHWC.empty(b, h, h, c, DEV)
            out = NHWC(x.t.clone())                 # FFC2 form: out = x + norm(...), in place over the residual
            pad = NHWC(torch.zeros(b, h + 2, h + 2, c, device=DEV))
            u = f1.pre_norm(ctx, x, y, None, xpad=xpad)
            assert (u is not None) == fused
            f1.norm(ctx, eng.bank, params, y, out, res=out, pad_out=pad, u=u)
            torch.cuda.synchronize()
            ctx.check_range()
            outs[fused] = (out.t.clone(), pad.t.clone())
    finally:
        ops.set_precision(prev)
    (o0, p0), (o1, p1) = outs[False], outs[True]
    assert torch.isfinite(o1).all()
    d = float((o0 - o1).abs().max())
    assert d <= TOL[prec], (prec, h, b, d)
    # the reflect-padded copy is the padded output exactly
    ref_pad = torch.nn.functional.pad(o1.permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect").permute(0, 2, 3, 1)
    assert torch.equal(p1, ref_pad)
    assert float((p0 - p1).abs().max()) <= TOL[prec]


def test_ffc_fused_off_in_f32(monkeypatch):
    """The exact-f32 arithmetic keeps the separate launches (the fused kernels are split-precision only)."""
    lnet, eng = _engine()
    f1 = eng.levels[1]["blocks"][0][0]
    prev = ops.set_precision("f32")
    try:
        assert not f1.fused()
    finally:
        ops.set_precision(prev)
    assert f1.fused() == (lnet.FUSED and f1.h in lnet.FUSED_LEVELS and ops.PRECISION in ("f16x3", "bf16x3"))


def test_lnet_fused_path_matches_reference(monkeypatch, golden):
    """The whole LNet (B = 2, 96x96) through the fused FFC kernels against the reference golden at the
    f16x3 bounds of tests/test_models_gpu.py."""
    from s2v_amd import models, synth
    from s2v_amd.engine import lnet
    from test_models_gpu import BAR, TOL, within
    monkeypatch.setattr(lnet, "FUSED", True)
    monkeypatch.setattr(lnet, "FUSED_LEVELS", (12, 24, 48))
    prev = ops.set_precision("f16x3")
    try:
        net = models.LNet()
        net.load_state_dict(synth_sd("lnet"), strict=True)
        g = golden("lnet_b2_96")
        mel, face, _ = synth.lipsync_inputs("golden.lnet", 2, 96)
        out = net.eval()(torch.from_numpy(mel).to(DEV), torch.from_numpy(face).to(DEV))
        eng = net._s2v_engines[str(out.device)][0]
        assert all(f.fused() for lv in eng.levels for blk in lv["blocks"] for f in blk)
    finally:
        ops.set_precision(prev)
    within(out, g["out"], BAR, "lnet fused bar")
    within(out, g["out"], TOL["f16x3"]["lnet"], "lnet fused")
