"""512x512 face enhancers on the device (SURVEY.md §8a GFPGAN / GPEN rows, config 5) against the
goldens the reference modules produced and against the CPU oracle.

Tolerances: fp32 throughout; outputs are unnormalised images (GFPGAN |x| <= ~35 with the
synthetic weights, GPEN |x| <= ~2.2).  Across ~40 conv layers the summation-order spread of fp32
is ~1e-5 relative per layer, so the bounds are 1e-3 relative to the tensor's max magnitude."""
import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import GFPGAN_KW, check_probe, max_abs, synth_sd
from s2v_amd import synth

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def gfpgan():
    from s2v_amd import models
    m = models.GFPGANv1Clean(**GFPGAN_KW)
    m.load_state_dict(synth_sd("gfpgan"), strict=True)
    return m.eval()


@pytest.fixture(scope="module")
def gpen():
    from s2v_amd import models
    m = models.FullGenerator(512, 512, 8, 2)
    m.load_state_dict(synth_sd("gpen"), strict=True)
    return m.eval()


@pytest.mark.parametrize("cfg", [
    dict(c=8, up=2, down=1, pad=(2, 1), hw=(9, 11)),          # ToRGB Upsample
    dict(c=3, up=2, down=1, pad=(2, 1), hw=(8, 8)),           # 3-channel skip (scalar path)
    dict(c=16, up=1, down=1, pad=(2, 2), hw=(13, 10)),        # encoder Blur
    dict(c=12, up=1, down=1, pad=(1, 1), hw=(17, 17)),        # blur after the transposed conv
    dict(c=4, up=1, down=2, pad=(1, 1), hw=(10, 10)),         # Downsample
])
def test_fir2d_matches_upfirdn2d(cfg):
    from oracle.enhancers import upfirdn2d
    from s2v_amd import ops
    from s2v_amd.ops import NHWC
    c, up, down, (p0, p1), (h, w) = cfg["c"], cfg["up"], cfg["down"], cfg["pad"], cfg["hw"]
    g = torch.Generator().manual_seed(c * 100 + up)
    x = torch.randn(2, c, h, w, generator=g)
    k = torch.tensor([1.0, 3.0, 3.0, 1.0])
    k = (k[None] * k[:, None]) / 64 * up * up
    ref = upfirdn2d(x, k, up=up, down=down, pad=(p0, p1))
    bias = torch.randn(c, generator=g)
    ref_act = torch.nn.functional.leaky_relu(1.5 * ref + bias[None, :, None, None], 0.2) * 2 ** 0.5
    ctx = ops.Ctx(DEV)
    xin = NHWC.empty(2, h, w, c + 4, DEV)                      # channel slice of a wider buffer
    ops.nchw_to_nhwc(ctx, x.to(DEV), xin.slice(4, c))
    for fused in (False, True):
        y = NHWC.empty(2, ref.shape[2], ref.shape[3], 2 * c, DEV)
        kw = dict(gain=1.5, bias=bias.to(DEV), act=ops.ACT_LRELU, alpha=0.2, post=2 ** 0.5) if fused else {}
        ops.fir2d(ctx, xin.slice(4, c), k.to(DEV), y.slice(c, c), up=up, down=down, pad0=(p0, p0), **kw)
        got = y.t[..., c:].permute(0, 3, 1, 2).cpu()
        assert max_abs(got, ref_act if fused else ref)[0] < 1e-5


def test_gfpgan_matches_reference(prec, gfpgan, golden):
    g = golden("gfpgan_b1_512")
    x = torch.from_numpy(synth.face_inputs("golden.gfpgan", 1)).to(DEV)
    img, rgbs = gfpgan(x, return_rgb=True, randomize_noise=False)
    assert max_abs(rgbs[0], g["rgb0"])[0] < 1e-3 * 51 and max_abs(rgbs[3], g["rgb3"])[0] < 1e-3 * 187
    check_probe(rgbs[6], g, "rgb6", atol=5e-3)
    err = check_probe(img, g, "out", atol=2e-3)
    print("gfpgan out max err", err)


@pytest.mark.parametrize("fold", [True, False])
def test_gfpgan_batch_vs_oracle_and_noise(gfpgan, fold, monkeypatch):
    """Both SFT forms: in the StyleConv epilogue (engine/gfpgan.py FOLD_SFT) and as its own pass."""
    from oracle import enhancers
    from s2v_amd.engine import gfpgan as eng
    monkeypatch.setattr(eng, "FOLD_SFT", fold)
    x = torch.from_numpy(synth.face_inputs("gfpgan.b2", 2))
    img, _ = gfpgan(x.to(DEV), return_rgb=False, randomize_noise=False)
    with torch.no_grad():
        ref, _, _ = enhancers.gfpgan_forward(synth_sd("gfpgan"), x, return_rgb=False)
    m, mean = max_abs(img, ref)
    assert m < 1e-3 * float(ref.abs().max()) and mean < 1e-4 * float(ref.abs().max()), (m, mean)
    a, _ = gfpgan(x.to(DEV), return_rgb=False)
    b, _ = gfpgan(x.to(DEV), return_rgb=False)
    assert torch.isfinite(a).all() and (a - b).abs().max() > 0       # fresh N(0,1) noise per call


def test_gpen_matches_reference(prec, gpen, golden):
    g = golden("gpen_b1_512")
    x = torch.from_numpy(synth.face_inputs("golden.gpen", 1)).to(DEV)
    img, lat = gpen(x, return_latents=True)
    assert lat.shape == (1, 16, 512)
    assert max_abs(lat[:, 0], g["latent"])[0] < 1e-4 * 7
    err = check_probe(img, g, "out", atol=1e-4)
    print("gpen out max err", err)


def test_gpen2048_matches_reference(prec, golden):
    """GPEN-BFR-2048 (the CLI's `enhancer` face GAN: FaceGAN(in_size=2048), inference.py:228-231;
    16/32-channel convs at 2048^2 and 1024^2) against the reference's own output probes."""
    from s2v_amd import models
    m = models.FullGenerator(2048, 512, 8, 2)
    m.load_state_dict(synth_sd("gpen2048"), strict=True)
    g = golden("gpen_b1_2048")
    x = torch.from_numpy(synth.face_inputs("golden.gpen2048", 1, 2048)).to(DEV)
    img, _ = m.eval()(x)
    assert img.shape == (1, 3, 2048, 2048)
    err = check_probe(img, g, "out", atol=1e-4)          # measured 2.8e-6 (f32) / 3.2e-5 (bf16x3)
    print(f"gpen2048 {prec} out max err {err:.2e} (|out| max {g['out_stats'][2]:.2f})")


@pytest.mark.parametrize("fold", [False, True])
def test_gpen_batch_vs_oracle(gpen, fold, monkeypatch):
    """Both noise-concat forms: a separate pass (the default) and the StyleConv epilogue's second output
    (engine/gpen.py FOLD_NOISE)."""
    from oracle import enhancers
    from s2v_amd.engine import gpen as eng
    monkeypatch.setattr(eng, "FOLD_NOISE", fold)
    x = torch.from_numpy(synth.face_inputs("gpen.b2", 2))
    img, none = gpen(x.to(DEV))
    assert none is None
    with torch.no_grad():
        ref, _, _ = enhancers.gpen_forward(synth_sd("gpen"), x)
    m, mean = max_abs(img, ref)
    assert m < 2e-3 and mean < 1e-4, (m, mean)
