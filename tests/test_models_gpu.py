"""End-to-end parity of the HIP models (s2v_amd.models, drop-in for reference models/) against
the reference outputs stored in tests/golden/ (and the CPU oracle for larger batches).

Two bars per output:
  * SURVEY.md §8d's fp32 per-pixel bar on what the caller consumes, for EVERY conv arithmetic mode:
    LNet / ENet [0,1]-scale outputs (ENet clamped to [0,1] as inference.py:267 does)
    max|d| <= 2e-3, mean|d| <= 1e-4;
  * a per-mode bound on the raw (unclamped) tensors at about twice the spread measured on MI355X
    (profiles/r02_precision.json; the reference's own fp32-vs-fp64 spread is 5e-4..7e-4).
    f32 (exact fp32 MFMA) and f16x3 (the default: 22-bit split operands) measure alike, e.g. ENet out
    2.3e-4 / 2.5e-4 max; bf16x3 (16-bit split operands) about 10x that.
"""

# per-mode raw bounds: (max, mean)
TOL = {
    "f32":    {"lnet": (1e-4, 1e-5), "logits": (1e-3, 1e-4), "enet": (6e-4, 6e-5), "low": (1e-4, 1e-5),
               "dnet": (2e-4, 2e-5), "flow": (3e-5, 5e-6)},
    "f16x3":  {"lnet": (1e-4, 1e-5), "logits": (1e-3, 1e-4), "enet": (6e-4, 6e-5), "low": (1e-4, 1e-5),
               "dnet": (2e-4, 2e-5), "flow": (3e-5, 5e-6)},
    "bf16x3": {"lnet": (1e-3, 1e-4), "logits": (5e-3, 3e-4), "enet": (5e-3, 5e-4), "low": (1e-3, 1e-4),
               "dnet": (2e-3, 1e-4), "flow": (3e-4, 5e-5)},
}
BAR = (2e-3, 1e-4)      # SURVEY.md §8d on [0,1] frames


def within(got, ref, bound, what):
    m, mean = max_abs(got, ref)
    assert m <= bound[0] and mean <= bound[1], (what, m, mean, bound)


def clamp01(t):
    t = t.detach().cpu() if isinstance(t, torch.Tensor) else torch.from_numpy(np.asarray(t))
    return t.double().clamp(0, 1)

import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import synth_sd, max_abs, check_probe
from s2v_amd import synth

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(name):
    from s2v_amd import models
    m = {"lnet": models.LNet, "enet": models.ENet, "dnet": models.DNet}[name]()
    m.load_state_dict(synth_sd(name), strict=True)
    return m.eval()


@pytest.fixture(scope="module")
def lnet():
    return _model("lnet")


@pytest.fixture(scope="module")
def enet():
    return _model("enet")


@pytest.fixture(scope="module")
def dnet():
    return _model("dnet")


def test_lnet_matches_reference(prec, lnet, golden):
    g = golden("lnet_b2_96")
    mel, face, _ = synth.lipsync_inputs("golden.lnet", 2, 96)
    out = lnet(torch.from_numpy(mel).to(DEV), torch.from_numpy(face).to(DEV))
    within(out, g["out"], BAR, "lnet bar")
    within(out, g["out"], TOL[prec]["lnet"], "lnet")


def test_lnet_intermediates(prec, lnet, golden):
    """Audio feature and pre-sigmoid logits through the engine directly."""
    from s2v_amd import ops
    from s2v_amd.ops import NHWC
    g = golden("lnet_b2_96")
    eng, ctx = lnet._engine(torch.device(DEV))
    mel, face, _ = synth.lipsync_inputs("golden.lnet", 2, 96)
    x6 = NHWC.empty(2, 96, 96, 6, DEV)
    ops.nchw_to_nhwc(ctx, torch.from_numpy(face).to(DEV), x6)
    out = NHWC.empty(2, 96, 96, 3, DEV)
    logits = NHWC.empty(2, 96, 96, 3, DEV)
    eng.forward(ctx, torch.from_numpy(mel).to(DEV), x6, out, logits=logits)
    lg = logits.t.permute(0, 3, 1, 2).cpu()
    within(lg, g["logits"], TOL[prec]["logits"], "logits")


def test_lnet_5d_input_fold(lnet):
    mel, face, _ = synth.lipsync_inputs("lnet.5d", 4, 96)
    m = torch.from_numpy(mel).to(DEV)
    f = torch.from_numpy(face).to(DEV)
    flat = lnet(m, f)
    # [B, T, 1, 80, 16] / [B, 6, T, H, W] with B=2, T=2 (LNet.py:124-127)
    m5 = torch.stack([m[:2], m[2:]], 1)
    f5 = torch.stack([f[:2], f[2:]], 2)
    out5 = lnet(m5, f5)
    assert out5.shape == (2, 3, 2, 96, 96)
    assert (out5[:, :, 0] - flat[:2]).abs().max() < 1e-6 and (out5[:, :, 1] - flat[2:]).abs().max() < 1e-6


def test_enet_matches_reference(prec, enet, golden):
    for size in (256, 384):
        g = golden(f"enet_b1_{size}")
        mel, face, gt = synth.lipsync_inputs(f"golden.enet{size}", 1, size)
        out, low = enet(torch.from_numpy(mel).to(DEV), torch.from_numpy(face).to(DEV), torch.from_numpy(gt).to(DEV))
        within(low, g["low"], BAR, ("low bar", size))
        within(low, g["low"], TOL[prec]["low"], ("low", size))
        if "out" in g.files:
            within(clamp01(out), clamp01(g["out"]), BAR, ("out clamped bar", size))
            within(out, g["out"], TOL[prec]["enet"], ("out", size))
        else:
            check_probe(out, g, "out", atol=TOL[prec]["enet"][0])


def test_enet_batch16_vs_oracle(prec, enet):
    """Full-size bench workload batch (B=16, 256x256 crops) against the CPU oracle on 2 frames of
    it, and batch-invariance (frames are independent) on the rest."""
    from oracle import nets
    mel, face, gt = synth.lipsync_inputs("enet.b16", 16, 256)
    out, low = enet(torch.from_numpy(mel).to(DEV), torch.from_numpy(face).to(DEV), torch.from_numpy(gt).to(DEV))
    sd = synth_sd("enet")
    with torch.no_grad():
        ro, rl = nets.enet_forward(sd, torch.from_numpy(mel[:2]), torch.from_numpy(face[:2]), torch.from_numpy(gt[:2]))
    within(clamp01(out[:2]), clamp01(ro), BAR, "b16 clamped bar")
    within(out[:2], ro, TOL[prec]["enet"], "b16 out")
    out2, _ = enet(torch.from_numpy(mel[8:10]).to(DEV), torch.from_numpy(face[8:10]).to(DEV),
                   torch.from_numpy(gt[8:10]).to(DEV))
    # a different batch size selects a different tile / split-K plan (fp32 summation order), so
    # only rounding-level agreement is expected
    assert (out2 - out[8:10]).abs().max() < 2e-3


def test_enet_polyphase_upsample_matches_upsample_pass():
    """The 200^2 -> 400^2 StyleConv as a depth-to-space polyphase conv with exact border lines
    (engine.enet.POLY_UP) against the upsample pass + conv, whole frames including every border
    pixel, with explicit StyleConv noise at a non-zero weight on both paths."""
    from s2v_amd.engine import enet as E
    mel, face, gt = synth.lipsync_inputs("enet.poly", 2, 256)
    args = [torch.from_numpy(a).to(DEV) for a in (mel, face, gt)]
    g = torch.Generator(device=DEV).manual_seed(5)
    noises = [torch.randn((2, 1, 100 * 2 ** (i // 2 + 1), 100 * 2 ** (i // 2 + 1)), generator=g, device=DEV)
              for i in range(4)]
    from s2v_amd import models
    sd = {k: (torch.full_like(v, 0.05) if k.startswith("style_convs.") and k.endswith(".weight") and v.numel() == 1
              else v) for k, v in synth_sd("enet").items()}
    model = models.ENet()
    model.load_state_dict(sd, strict=True)
    model.eval()
    outs = {}
    for poly in (True, False):
        prev = E.POLY_UP
        E.POLY_UP = poly
        try:
            outs[poly] = model(*args, noises=noises)[0]
        finally:
            E.POLY_UP = prev
    err = (outs[True] - outs[False]).abs()
    assert err.max() < 2e-3 and err.mean() < 2e-5, (float(err.max()), float(err.mean()))


def test_enet_5d_input_fold(enet):
    """ENet.forward folds [B, C, T, H, W] face / gt and [B, T, 1, 80, 16] audio into the batch and
    unfolds the outputs (ENet.py:87-91, :131-137)."""
    mel, face, gt = synth.lipsync_inputs("enet.5d", 4, 256)
    m, f, g = (torch.from_numpy(a).to(DEV) for a in (mel, face, gt))
    out, low = enet(m, f, g)
    m5 = torch.stack([m[:2], m[2:]], 1)
    f5, g5 = torch.stack([f[:2], f[2:]], 2), torch.stack([g[:2], g[2:]], 2)
    out5, low5 = enet(m5, f5, g5)
    # low_res_img is nearest-resized to the output size before the unfold (ENet.py:134)
    assert out5.shape == (2, 3, 2, 384, 384) and low5.shape == (2, 3, 2, 384, 384)
    up = torch.nn.functional.interpolate(low.cpu(), (384, 384))
    for t in range(2):
        assert (out5[:, :, t] - out[2 * t: 2 * t + 2]).abs().max() < 2e-3
        assert (low5[:, :, t].cpu() - up[2 * t: 2 * t + 2]).abs().max() < 1e-5


def test_dnet_matches_reference(prec, dnet, golden):
    for size, batch in ((128, 2), (256, 1)):
        g = golden(f"dnet_b{batch}_{size}")
        src, coeff = synth.dnet_inputs(f"golden.dnet{size}", batch, size)
        out = dnet(torch.from_numpy(src).to(DEV), torch.from_numpy(coeff).to(DEV))
        within(out["flow_field"], g["flow"], TOL[prec]["flow"], "flow")
        for k in ("warp_image", "fake_image"):
            if k in g.files:
                within(out[k], g[k], TOL[prec]["dnet"], k)
            else:
                check_probe(out[k], g, k, atol=TOL[prec]["dnet"][0])


def test_dnet_warp_stage(dnet):
    src, coeff = synth.dnet_inputs("dnet.stage", 1, 128)
    full = dnet(torch.from_numpy(src).to(DEV), torch.from_numpy(coeff).to(DEV))
    warp = dnet(torch.from_numpy(src).to(DEV), torch.from_numpy(coeff).to(DEV), stage="warp")
    assert "fake_image" not in warp
    assert torch.equal(warp["warp_image"], full["warp_image"])


def test_cpu_inputs_fail_loudly(lnet):
    mel, face, _ = synth.lipsync_inputs("cpu", 1, 96)
    with pytest.raises(RuntimeError):
        lnet(torch.from_numpy(mel), torch.from_numpy(face))
