"""GFPGANer's restore composition on the device (gfpgan/utils.py:97-143, facexlib 0.2.5
FaceRestoreHelper) against the CPU restatement oracle/restore.py.

Bars: the uint8 alignment warp with the gray border, tensor2img, the square-mask erosions and the
fp32 paste-back blend are BIT-EXACT (the restatement's operation order, no FMA contraction); the
erosion area is an fp64 sum on the device vs numpy's fp32 pairwise sum (relative 1e-6; only
int(sqrt(area)) // 20 is used).  GFPGANv1Clean itself is compared with its oracle in
test_enhancers_gpu.py; the end-to-end test feeds the device's network output to the restatement.
Parity UNPINNED (facexlib and OpenCV are absent from the image)."""
import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import GFPGAN_KW, synth_sd
from oracle import face as OF
from oracle import restore as OR

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rng_u8(seed, shape):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def _sim(angle, scale, tx, ty):
    c, s = np.cos(angle) * scale, np.sin(angle) * scale
    return np.array([[c, -s, tx], [s, c, ty]])


def _ctx():
    from s2v_amd import face
    return face._ctx(DEV)


def test_align_warp_with_gray_border_bit_exact():
    """align_warp_face's warpAffine(img, affine, (512, 512), borderValue=(135, 133, 132)) for several
    faces of one frame (one launch, source image pitch 0)."""
    from s2v_amd import _lib, restore
    import ctypes
    img = rng_u8(1, (150, 170, 3))
    Ms = [_sim(0.2, 2.9, -60.0, -20.0), _sim(-0.5, 4.1, 40.0, -300.0), _sim(0.0, 1.0, 0.0, 0.0)]
    n, S = len(Ms), 96
    out = torch.empty((n, S, S, 3), dtype=torch.uint8, device=DEV)
    src = torch.from_numpy(img).to(DEV)
    md = torch.from_numpy(np.stack(Ms).reshape(n, 6)).to(DEV)
    ctx = _ctx()
    border = (ctypes.c_double * 3)(*restore.BORDER_GRAY)
    _lib.check(ctx.lib.s2v_warp_affine_border(src.data_ptr(), n, 150, 170, 3, 170 * 3, 0, 0, md.data_ptr(),
                                              out.data_ptr(), S, S, S * 3, S * S * 3, border, ctx.stream), "warp")
    got = out.cpu().numpy()
    for i, M in enumerate(Ms):
        exp = OF.warp_affine(img, M, (S, S), border_value=np.array(OR.BORDER_GRAY))
        assert np.array_equal(got[i], exp), (i, int((got[i] != exp).sum()))
    assert (got[1] == np.array(OR.BORDER_GRAY, np.uint8)).all(axis=-1).any()   # the gray border is there


def test_tensor2img_bit_exact():
    y = np.random.default_rng(2).uniform(-1.3, 1.3, (2, 3, 20, 24)).astype(np.float32)
    y[0, 0, 0, :4] = [-1.0, 1.0, 0.0, 1.0 / 255.0 - 1.0]
    out = torch.empty((2, 20, 24, 3), dtype=torch.uint8, device=DEV)
    ctx = _ctx()
    assert ctx.lib.s2v_tensor2img_u8(torch.from_numpy(y).to(DEV).data_ptr(), 2, 20, 24, out.data_ptr(),
                                     ctx.stream) == 0
    got = out.cpu().numpy()
    for i in range(2):
        assert np.array_equal(got[i], OR.tensor2img(y[i]))


INVS = [OR.invert_affine_transform(_sim(0.25, 2.7, -55.0, -30.0)),       # a 512 crop of a rotated face
        OR.invert_affine_transform(_sim(-0.1, 4.0, -200.0, -150.0)),
        OR.invert_affine_transform(_sim(0.0, 1.0, -20.0, -10.0))]


@pytest.mark.parametrize("mi", range(len(INVS)))
def test_restore_mask_erosion_and_area(mi):
    from s2v_amd import _lib, face
    H, W, S = 260, 300, 512
    inv = INVS[mi]
    E = torch.empty((H, W), device=DEV)
    area = torch.empty(1 + 512, dtype=torch.float64, device=DEV)
    ctx = _ctx()
    md = face._mats(inv, DEV)
    _lib.check(ctx.lib.s2v_restore_mask(md.data_ptr(), S, H, W, 0, 0, H, W, E.data_ptr(), area.data_ptr(),
                                        ctx.stream), "mask")
    exp = OR.erode(OF.warp_affine(np.ones((S, S), np.float32), inv, (W, H)), 2)
    got = E.cpu().numpy()
    assert np.array_equal(got, exp), np.abs(got - exp).max()
    ref = float(np.sum(exp))
    assert ref > 100 and abs(area[0].item() - ref) <= 1e-6 * ref


@pytest.mark.parametrize("k", [1, 3, 4, 10, 31])
def test_erode_rect_bit_exact(k):
    from s2v_amd import _lib
    x = np.random.default_rng(k).random((70, 95)).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    y, ws = torch.empty_like(xd), torch.empty_like(xd)
    ctx = _ctx()
    _lib.check(ctx.lib.s2v_erode_rect_f32(xd.data_ptr(), 70, 95, k, y.data_ptr(), ws.data_ptr(), ctx.stream), "erode")
    assert np.array_equal(y.cpu().numpy(), OR.erode(x, k))


def _helper(face_det=None):
    from s2v_amd import restore
    return restore.FaceRestoreHelper(1, face_size=512, device=DEV, face_det=face_det or _NoDetector())


class _NoDetector:
    def detect_faces(self, img, conf_threshold=0.8):
        raise AssertionError("not used")


@pytest.mark.parametrize("nfaces", [1, 2, 3])
def test_paste_faces_to_input_image_bit_exact(nfaces):
    """paste_faces_to_input_image on given restored faces / inverse affines: one face (uint8 -> uint8),
    two overlapping faces (the second blends onto the fp32 result of the first) and a third whose crop
    covers the whole frame (mask window clipped to the frame: the blur's reflect-101 edges)."""
    img = rng_u8(5, (260, 300, 3))
    restored = [rng_u8(6 + i, (512, 512, 3)) for i in range(nfaces)]
    inv = INVS[:nfaces]
    fh = _helper()
    fh.read_image(img)
    fh.restored_faces = [torch.from_numpy(f).to(DEV) for f in restored]
    fh.inverse_affine_matrices = list(inv)
    trace = []
    got = fh.paste_faces_to_input_image(trace=trace).cpu().numpy()
    otrace = []
    exp = OR.paste_faces(img, restored, inv, (512, 512), otrace)
    for a, b in zip(trace, otrace):
        assert a["w_edge"] == b["w_edge"] > 0
        y0, x0, wh, ww = a["window"]
        for key in ("soft", "erosion"):                  # the windowed masks, zero elsewhere, = the full frame's
            full = np.zeros_like(b[key])
            full[y0: y0 + wh, x0: x0 + ww] = a[key].cpu().numpy()
            assert np.array_equal(full, b[key]), key
    assert np.array_equal(got, exp), int((got != exp).sum())
    assert not np.array_equal(got, img)


def test_paste_without_faces_returns_the_input():
    img = rng_u8(9, (40, 50, 3))
    fh = _helper()
    fh.read_image(img)
    assert np.array_equal(fh.paste_faces_to_input_image().cpu().numpy(), img)


# ----------------------------------------------------------------------------- end to end
class _FixedFaces:
    """facexlib detect_faces rows for a frame: faces whose landmarks are the FFHQ template under known
    similarities (plus a side face with eye distance < 5 that the helper drops)."""

    def __init__(self, h, w):
        self.calls = []
        tpl = OR.FFHQ_TEMPLATE_512
        rows = []
        for (ang, sc, cx, cy, score) in ((0.15, 0.3, w * 0.45, h * 0.55, 0.999), (-0.3, 0.18, w * 0.85, h * 0.2, 0.98),
                                         (0.0, 0.004, w * 0.5, h * 0.5, 0.99)):
            M = _sim(ang, sc, 0.0, 0.0)
            p = (tpl - 256.0) @ M[:, :2].T + np.array([cx, cy])
            box = [p[:, 0].min() - 20 * sc, p[:, 1].min() - 40 * sc, p[:, 0].max() + 20 * sc, p[:, 1].max() + 30 * sc]
            rows.append(box + [score] + list(p.reshape(-1)))
        self.rows = np.array(rows, np.float32)

    def detect_faces(self, img, conf_threshold=0.8):
        self.calls.append(conf_threshold)
        return self.rows.copy()


@pytest.fixture(scope="module")
def gfpgan():
    from s2v_amd import models
    m = models.GFPGANv1Clean(**GFPGAN_KW)
    m.load_state_dict(synth_sd("gfpgan"), strict=True)
    return m.eval()


@pytest.mark.parametrize("center", [True, False])
def test_gfpganer_enhance_matches_the_restatement(gfpgan, center):
    """GFPGANer.enhance(ff, has_aligned=False, only_center_face=center, paste_back=True) (inference.py:300):
    landmarks -> LMEDS fit -> gray-border warp (bit-exact), img2tensor + GFPGAN + tensor2img (the
    device network's output through the restatement's tensor2img: bit-exact), paste-back (bit-exact)."""
    from s2v_amd import restore
    H, W = 240, 320
    img = rng_u8(31, (H, W, 3))
    det = _FixedFaces(H, W)
    r = restore.GFPGANer(upscale=1, device=DEV, net=gfpgan, face_det=det, randomize_noise=False)
    cropped, restored, out = r.enhance(img, has_aligned=False, only_center_face=center, paste_back=True)
    assert det.calls == [0.97]
    assert len(cropped) == len(restored) == (1 if center else 2)        # the tiny face is dropped
    # the device's batch: the same img2tensor launch and network call GFPGANer._restore makes
    u8 = torch.stack(cropped).contiguous()
    X = torch.empty((len(cropped), 3, 512, 512), device=DEV)
    ctx = _ctx()
    assert ctx.lib.s2v_u8_to_gan(u8.data_ptr(), len(cropped), 512, 512, X.data_ptr(), ctx.stream) == 0
    Y = gfpgan(X, return_rgb=False, randomize_noise=False)[0].cpu().numpy()
    X = X.cpu().numpy()
    calls = iter(range(len(cropped)))

    def fake_gfpgan(x):
        i = next(calls)
        assert np.array_equal(x, X[i])                 # img2tensor + normalize restated bit for bit
        return Y[i]

    otrace = {}
    ocrop, orest, oout = OR.enhance(img, detect_faces=det.detect_faces, gfpgan=fake_gfpgan,
                                    only_center_face=center, trace=otrace)
    for a, b in zip(cropped, ocrop):
        assert np.array_equal(a.cpu().numpy(), b)
    for a, b in zip(r.face_helper.affine_matrices, otrace["affines"]):
        assert np.array_equal(a, b)
    for a, b in zip(restored, orest):
        assert np.array_equal(a.cpu().numpy(), b)
    got = out.cpu().numpy()
    assert np.array_equal(got, oout), int((got != oout).sum())


def test_gfpganer_aligned_and_no_paste(gfpgan):
    from s2v_amd import restore
    img = rng_u8(32, (128, 128, 3))
    r = restore.GFPGANer(upscale=1, device=DEV, net=gfpgan, face_det=_NoDetector(), randomize_noise=False)
    cropped, restored, out = r.enhance(img, has_aligned=True)
    assert out is None and len(cropped) == len(restored) == 1 and cropped[0].shape == (512, 512, 3)
    H, W = 200, 260
    r2 = restore.GFPGANer(upscale=1, device=DEV, net=gfpgan, face_det=_FixedFaces(H, W), randomize_noise=False)
    c2, r2f, out2 = r2.enhance(rng_u8(33, (H, W, 3)), only_center_face=True, paste_back=False)
    assert out2 is None and len(c2) == len(r2f) == 1


def test_retinaface_detect_faces_matches_facexlib_postprocess():
    """RetinaFaceDetector.detect_faces: the device decode + threshold, then facexlib's sort / NMS /
    row layout, against the restatement over the same device head outputs."""
    from s2v_amd import face, models, restore
    m = models.RetinaFace()
    m.load_state_dict(synth_sd("retinaface"), strict=True)
    det = restore.RetinaFaceDetector(device=DEV, net=m.eval())
    img = rng_u8(41, (150, 190, 3))
    maps = det.det.head_maps(torch.from_numpy(img).to(DEV))
    loc, conf, lms = (t[0].cpu() for t in models.retina_outputs(face._ctx(DEV), maps, 150, 190))
    v = np.unique(conf[:, 1].numpy())
    thr = float(v[max(0, len(v) - 1 - max(1, int(len(v) * 0.03)))])
    rows = det.detect_faces(img, thr)
    priors = OF.prior_box((150, 190))
    boxes = (OF.decode(loc, priors, OF.CFG["variance"]) * torch.Tensor([190, 150, 190, 150])).numpy()
    lm = (OF.decode_landm(lms, priors, OF.CFG["variance"]) * torch.Tensor([190, 150] * 5)).numpy()
    scores = conf.numpy()[:, 1]
    inds = np.where(scores > np.float32(thr))[0]
    exp = OR.detect_faces_post(boxes[inds], scores[inds], lm[inds])
    assert rows.shape == exp.shape and len(rows) > 0
    np.testing.assert_allclose(rows, exp, rtol=3e-7, atol=1e-4)
