"""Mouth-region post-process on the device (inference.py:302-313) against the CPU
restatement (oracle/post.py, oracle/parse.py) and the ParseNet goldens from the reference module.

Bars: the pyramid / resize / mask / conversion kernels are compared BIT-EXACT with the NumPy
restatement (same integer arithmetic; float ops rounded one by one in the same order).  ParseNet is
floating point: logits within 1e-4 (f32) / 1e-3 (bf16x3) of max|logit| (about 40 conv layers, the
reference's own fp32-vs-fp64 spread is ~1e-4 relative), and the argmax equal wherever the oracle's
top-2 margin exceeds that bound (near-ties may flip)."""
import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import check_probe, max_abs, parsenet_sd
from oracle import parse as OPARSE
from oracle import post as OP
from s2v_amd import synth

pytestmark = pytest.mark.gpu
DEV = "cuda"
ATOL = {"f32": 1e-4, "bf16x3": 1e-3, "f16x3": 1e-4}


def rng_u8(seed, shape):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def smooth_mask(seed, h, w):
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w] / np.float32(max(h, w))
    m = 0.5 + 0.5 * np.sin(7 * xx + 3 * g.random()) * np.cos(5 * yy + 3 * g.random())
    m[g.random((h, w)) < 0.05] = 1.0
    return m.astype(np.float32)


@pytest.mark.parametrize("n,h,w,c,levels", [(2, 64, 96, 3, 1), (2, 64, 96, 3, 4), (1, 96, 64, 3, 6),
                                            (1, 512, 512, 3, 10), (3, 32, 32, 1, 6)])
def test_laplacian_blend_bit_exact(n, h, w, c, levels):
    from s2v_amd import post
    A = rng_u8(1, (n, h, w, c))
    B = rng_u8(2, (n, h, w, c))
    M = np.stack([smooth_mask(3 + i, h, w) for i in range(n)])
    got = post.laplacian_pyramid_blending_with_mask(A if c > 1 else A[..., 0:1], B, M, levels).cpu().numpy()
    for i in range(n):
        ref = OP.laplacian_blend(A[i], B[i], M[i], levels)
        assert np.array_equal(got[i].reshape(ref.shape), ref), f"image {i}: max diff {np.abs(got[i].reshape(ref.shape) - ref).max()}"
    clipped = post.laplacian_pyramid_blending_with_mask(A, B, M, levels, clip=True).cpu().numpy()
    assert np.array_equal(clipped, np.clip(got, 0, 255))


def test_laplacian_blend_rejects_ragged_pyramids():
    from s2v_amd import post
    from s2v_amd._lib import S2VError
    a = torch.zeros((32, 24, 3), dtype=torch.uint8, device=DEV)
    with pytest.raises(S2VError):
        post.laplacian_pyramid_blending_with_mask(a, a, torch.zeros((32, 24), device=DEV), 6)


@pytest.mark.parametrize("src,dst", [((37, 53), (512, 512)), ((512, 512), (21, 17)), ((300, 200), (200, 300)),
                                     ((5, 5), (5, 5))])
def test_resize_linear_bit_exact(src, dst):
    from s2v_amd import post
    img = rng_u8(sum(src), src + (3,))
    H, W = dst
    assert np.array_equal(post.resize_linear(torch.from_numpy(img).to(DEV), (W, H)).cpu().numpy(),
                          OP.resize_linear(img, (W, H)))
    f = (np.random.default_rng(7).random(src, dtype=np.float32) * 300 - 20).astype(np.float32)
    fd = torch.from_numpy(f).to(DEV)
    assert np.array_equal(post.resize_linear(fd, (W, H)).cpu().numpy(), OP.resize_linear(f, (W, H)))
    fc = np.clip(f, 0, 255)
    got = post.resize_linear(torch.from_numpy(fc).to(DEV), (W, H), mode=post.RS_F32_TO_U8).cpu().numpy()
    assert np.array_equal(got, OP.resize_linear(fc, (W, H)).astype(np.uint8))


def test_resize_roi_and_mask_paste():
    from s2v_amd import post
    frame = rng_u8(11, (120, 160, 3))
    fd = torch.from_numpy(frame).to(DEV)
    y1, y2, x1, x2 = 17, 90, 33, 121
    crop = post.resize_linear(fd[y1:y2, x1:x2], (512, 512)).cpu().numpy()
    assert np.array_equal(crop, OP.resize_linear(np.ascontiguousarray(frame[y1:y2, x1:x2]), (512, 512)))
    tmp = np.zeros((512, 512), np.uint8)
    tmp[100:380, 50:460] = 255
    tmp[380:390] = 254
    full = torch.zeros((120, 160), device=DEV)
    post.resize_linear(torch.from_numpy(tmp).to(DEV), (x2 - x1, y2 - y1), out=full[y1:y2, x1:x2],
                       mode=post.RS_U8_EQ255)
    assert np.array_equal(full.cpu().numpy(), OP.mouth_mask_full(tmp, (120, 160), (y1, y2, x1, x2)))


def test_parse_mask_and_img2tensor():
    from s2v_amd import ops, post
    from s2v_amd.ops import NHWC
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(2, 19, 33, 47, generator=g)
    x = NHWC(logits.permute(0, 2, 3, 1).contiguous().to(DEV))
    got = post.parse_mask(x, post.MOUTH_MM).cpu().numpy()
    ref = np.stack(OP.tenor2mask(logits.numpy(), OP.MOUTH_MM))
    assert np.array_equal(got, ref)
    img = rng_u8(5, (2, 9, 13, 3))
    parser = post.FaceParse.__new__(post.FaceParse)
    parser.device = torch.device(DEV)
    parser.faceparse = type("E", (), {"_engine": lambda self, d: (None, ops.Ctx(d))})()
    x4 = parser.img2tensor_nhwc(torch.from_numpy(img).to(DEV))
    for i in range(2):
        assert np.array_equal(x4.t[i, ..., :3].cpu().numpy(), OP.img2tensor(img[i])[0].transpose(1, 2, 0))
    assert (x4.t[..., 3] == 0).all()


@pytest.fixture(scope="module")
def parsenets():
    from s2v_amd import models
    from s2v_amd.models.parse_arch import face_parse_net
    nets = {}
    for size in (128, 512):
        m = models.ParseNet(**face_parse_net(size))
        m.load_state_dict(parsenet_sd(size), strict=True)
        nets[size] = m.eval()
    return nets


def _argmax_agrees(mask, ref_logits, atol):
    ref = ref_logits.double()
    top2 = ref.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 2 * atol
    same = mask.argmax(1).cpu() == ref.argmax(1)
    assert bool(same[clear].all()), f"{int((~same[clear]).sum())} clear-margin pixels disagree"
    assert float(same.float().mean()) > 0.999


def test_parsenet_matches_reference(prec, parsenets, golden):
    for size, batch in ((128, 2), (512, 1)):
        g = golden(f"parsenet_b{batch}_{size}")
        x = torch.from_numpy(synth.face_inputs(f"golden.parsenet{size}", batch, size)).to(DEV)
        mask, img = parsenets[size](x)
        if size == 128:
            scale = float(np.abs(g["mask"]).max())
            atol = ATOL[prec] * scale
            assert max_abs(mask, g["mask"])[0] < atol and max_abs(img, g["img"])[0] < atol
            _argmax_agrees(mask, torch.from_numpy(g["mask"]), atol)
        else:
            atol = ATOL[prec] * float(g["mask_stats"][2])
            check_probe(mask, g, "mask", atol=atol)
            check_probe(img, g, "img", atol=ATOL[prec] * float(g["img_stats"][2]))
            assert float((mask.argmax(1).cpu().numpy() == g["argmax"]).mean()) > 0.999


def test_face_parse_process_vs_oracle(parsenets):
    from s2v_amd import post
    parser = post.FaceParse(net=parsenets[512])
    face = rng_u8(21, (200, 180, 3))
    got = parser.process(face, post.MOUTH_MM)[0]
    im512 = OP.resize_linear(face, (512, 512))
    logits = OPARSE.mask_logits(parsenet_sd(512), im512)
    ref = OP.tenor2mask(logits.numpy(), OP.MOUTH_MM)[0]
    assert got.shape == (512, 512) and float((got == ref).mean()) > 0.999
    t = parser.process_tensor(torch.rand(2, 3, 96, 80, device=DEV))
    assert t.shape == (1, 2, 512, 512) and t.dtype == torch.int64
    assert set(torch.unique(t).tolist()) <= {0, 255}


def test_mouth_blend_compose_bit_exact_and_full_run(parsenets):
    from s2v_amd import post
    H, W = 256, 320
    restored = rng_u8(31, (2, H, W, 3))
    ff = rng_u8(32, (2, H, W, 3))
    coords = [(40, 200, 60, 250), (0, 256, 100, 320)]
    mb = post.MouthBlend(post.FaceParse(net=parsenets[512]))
    tmp = np.zeros((2, 512, 512), np.uint8)
    tmp[:, 250:400, 120:400] = 255
    got = mb.compose(torch.from_numpy(restored).to(DEV), torch.from_numpy(ff).to(DEV),
                     torch.from_numpy(tmp).to(DEV), coords).cpu().numpy()
    for i in range(2):
        full = OP.mouth_mask_full(tmp[i], (H, W), coords[i])
        assert np.array_equal(got[i], OP.blend_frame(restored[i], ff[i], full)), i
    out = mb.run_batch(torch.from_numpy(restored).to(DEV), torch.from_numpy(ff).to(DEV), coords).cpu().numpy()
    assert out.shape == (2, H, W, 3) and out.dtype == np.uint8
