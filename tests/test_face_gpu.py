"""Face detection / alignment / FaceEnhancement on the device (face_enhancement.py:91-193)
against the CPU restatement (oracle/face.py, pinned to the reference goldens in test_face_host.py).

Bars:
* integer / byte kernels (uint8 warpAffine, filter2D, tensor2img, the paste-back and the blends
  composed on identical inputs): BIT-EXACT;
* float kernels evaluated in the restatement's operation order (fp32 / fp64 warpAffine, the fp64
  Gaussian blurs of mask_postprocess, img2tensor): BIT-EXACT as well (no FMA contraction on either
  side); the test states a 0 tolerance and fails on any difference;
* RetinaFace-R50 (floating point through ~70 conv layers): loc / conf / landms within 1e-3 of the
  output scale of the fp32 CPU oracle in every conv arithmetic mode; the device decode + threshold
  + NMS equal to the oracle's post-processing of the same device head outputs (decoded values
  within 2 ulp: expf vs torch's CPU exp).
The composition tests inject the device's network outputs (detections, GPEN faces, parse masks, SR
frame) into oracle.face.enhance_process: every network is checked against its own oracle elsewhere
(test_enhancers_gpu / test_post_gpu / test_sr_gpu and the RetinaFace test here).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import s2v_import  # noqa: F401
from helpers import parsenet_sd, rrdb_sd, synth_sd
from oracle import face as OF
from oracle import post as OP

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rng_u8(seed, shape):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def _rot(angle, scale, tx, ty):
    c, s = np.cos(angle) * scale, np.sin(angle) * scale
    return np.array([[c, -s, tx], [s, c, ty]])


WARPS = [_rot(0.0, 1.0, 0.0, 0.0), _rot(0.3, 0.8, 12.3, -4.7), _rot(-1.1, 2.3, 40.0, 7.25), _rot(2.9, 0.37, 80.0, 90.0),
         np.array([[1.0, 0.0, -0.5], [0.0, 1.0, 0.25]]), _rot(0.05, 1.0, -300.0, 10.0)]


@pytest.mark.parametrize("mi", range(len(WARPS)))
@pytest.mark.parametrize("dtype", ["u8", "f32", "f64"])
def test_warp_affine_bit_exact(mi, dtype):
    from s2v_amd import face
    M = WARPS[mi]
    if dtype == "u8":
        src = rng_u8(mi, (57, 83, 3))
    else:
        src = np.random.default_rng(mi).random((57, 83)).astype(np.float32 if dtype == "f32" else np.float64)
    for dsize in ((83, 57), (64, 40), (130, 97)):
        got = face.warp_affine(torch.from_numpy(src).to(DEV), M, dsize).cpu().numpy()
        exp = OF.warp_affine(src, M, dsize)
        assert got.dtype == exp.dtype and got.shape == exp.shape
        assert np.array_equal(got, exp), (dtype, mi, dsize, np.abs(got.astype(np.float64) - exp).max())


def test_warp_affine_batch_and_roi():
    from s2v_amd import face
    src = rng_u8(7, (3, 40, 50, 3))
    Ms = np.stack(WARPS[1:4])
    got = face.warp_affine(torch.from_numpy(src).to(DEV), Ms, (45, 35)).cpu().numpy()
    for i in range(3):
        assert np.array_equal(got[i], OF.warp_affine(src[i], Ms[i], (45, 35)))
    frame = torch.zeros((60, 70, 3), dtype=torch.uint8, device=DEV)
    face.warp_affine(torch.from_numpy(src[0]).to(DEV), Ms[0], (30, 20), out=frame[5:25, 10:40])
    f = frame.cpu().numpy()
    assert np.array_equal(f[5:25, 10:40], OF.warp_affine(src[0], Ms[0], (30, 20))) and f[:5].sum() == 0


def test_mask_postprocess_and_blur_bit_exact():
    from s2v_amd import face
    g = np.random.default_rng(3)
    m = np.zeros((512, 512), np.uint8)
    m[100:400, 120:380] = 255
    m[g.random((512, 512)) < 0.02] = 255
    got = face.mask_postprocess(torch.from_numpy(m).to(DEV)).cpu().numpy()
    exp = OF.mask_postprocess(m / 255.)
    assert got.dtype == np.float32 and np.array_equal(got, exp), np.abs(got - exp).max()
    x = g.random((70, 90))
    got = face.gaussian_blur(torch.from_numpy(x).to(DEV), 0, 1.0).cpu().numpy()
    assert got.dtype == np.float64 and np.array_equal(got, OF.gaussian_blur(x, 0, 1.0))
    x32 = x.astype(np.float32)
    got = face.gaussian_blur(torch.from_numpy(x32).to(DEV), 31, 4.0).cpu().numpy()
    assert np.array_equal(got, OF.gaussian_blur(x32, 31, 4.0))


def test_mask_sharp_keeps_the_zeroed_border():
    """face_enhancement.py:144-150: mask_postprocess zeroes a 26-px border of mask_sharp in place
    before mask_sharp is resized and warped; the device's mask_sharp (s2v_u8_div255_f64_border) must
    carry that border too, for a parse mask that reaches the crop edge."""
    from s2v_amd import _lib, face
    g = np.random.default_rng(7)
    m = np.zeros((512, 512), np.uint8)
    m[g.random((512, 512)) < 0.5] = 255
    m[:, :3] = 255                                    # face region touching every crop edge
    m[-2:, :] = 255
    exp = m / 255.
    OF.mask_postprocess(exp)                          # mutates exp like the reference's mask_sharp
    assert exp[:26].max() == 0 and exp[:, -26:].max() == 0 and exp[26:-26, 26:-26].max() == 1.0
    src = torch.from_numpy(m).to(DEV)
    got = torch.empty((512, 512), dtype=torch.float64, device=DEV)
    lib = _lib.load()
    _lib.check(lib.s2v_u8_div255_f64_border(src.data_ptr(), 512, 512, face.MASK_BORDER, got.data_ptr(),
                                            torch.cuda.current_stream().cuda_stream), "div255_border")
    assert np.array_equal(got.cpu().numpy(), exp)


def test_filter2d_and_gan_conversions_bit_exact():
    from s2v_amd import face
    img = rng_u8(4, (33, 47, 3))
    got = face.filter2d_smooth(torch.from_numpy(img).to(DEV)).cpu().numpy()
    assert np.array_equal(got, OF.filter2d_u8(img, OF.SMALL_FACE_KERNEL))
    lib = face._ctx(DEV).lib
    ctx = face._ctx(DEV)
    faces = rng_u8(5, (2, 16, 16, 3))
    x = torch.empty((2, 3, 16, 16), device=DEV)
    assert lib.s2v_u8_to_gan(torch.from_numpy(faces).to(DEV).data_ptr(), 2, 16, 16, x.data_ptr(), ctx.stream) == 0
    ref = ((torch.from_numpy(faces) / 255. - 0.5) / 0.5).permute(0, 3, 1, 2).flip(1)    # face_gan.py:44-49
    assert torch.equal(x.cpu(), ref)
    y = torch.from_numpy(np.random.default_rng(6).uniform(-1.3, 1.3, (2, 3, 16, 16)).astype(np.float32))
    out = torch.empty((2, 16, 16, 3), dtype=torch.uint8, device=DEV)
    assert lib.s2v_gan_to_u8(y.to(DEV).data_ptr(), 2, 16, 16, out.data_ptr(), ctx.stream) == 0
    t = (y * 0.5 + 0.5).permute(0, 2, 3, 1).flip(3)                                          # face_gan.py:51-59
    exp = (np.clip(t.numpy(), 0, 1) * 255.0).astype(np.uint8)
    assert np.array_equal(out.cpu().numpy(), exp)


def test_maxpool_matches_torch():
    from s2v_amd import face
    x = torch.randn(2, 17, 23, 64)
    y = torch.empty(2, 9, 12, 64, device=DEV)
    ctx = face._ctx(DEV)
    assert ctx.lib.s2v_maxpool2d_nhwc(x.to(DEV).data_ptr(), 2, 17, 23, 64, 3, 2, 1, y.data_ptr(), 9, 12, ctx.stream) == 0
    ref = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(y.cpu(), ref)


# ----------------------------------------------------------------------------- RetinaFace
@pytest.fixture(scope="module")
def retina():
    from s2v_amd import models
    m = models.RetinaFace()
    m.load_state_dict(synth_sd("retinaface"), strict=True)
    return m.eval()


def _retina_input(seed, h, w):
    img = rng_u8(seed, (h, w, 3))
    x = torch.from_numpy(np.float32(img) - np.array([104, 117, 123], np.float32)).permute(2, 0, 1)[None]
    return img, x.contiguous()


def test_retinaface_forward_matches_oracle(retina, prec):
    img, x = _retina_input(11, 150, 190)
    loc, conf, lms = retina(x.to(DEV))
    with torch.no_grad():
        rl, rc, rm = OF.retinaface_forward(synth_sd("retinaface"), x)
    P = sum(2 * (-(-150 // s)) * (-(-190 // s)) for s in (8, 16, 32))
    assert loc.shape == (1, P, 4) and conf.shape == (1, P, 2) and lms.shape == (1, P, 10)
    for got, ref in ((loc, rl), (conf, rc), (lms, rm)):
        d = (got.cpu() - ref).abs().max().item()
        assert d <= 1e-3 * max(1.0, ref.abs().max().item()), (prec, d)
    assert torch.allclose(conf.sum(-1).cpu(), torch.ones(1, P), atol=1e-6)


def _threshold(conf, frac):
    """A confidence threshold passing about ``frac`` of the anchors (at least one): synthetic weights
    saturate many scores, so pick a value strictly below a distinct score."""
    v = np.unique(conf[:, 1].numpy())
    return float(v[max(0, len(v) - 1 - max(1, int(len(v) * frac)))])


def test_retinaface_detect_matches_oracle_postprocess(retina):
    from s2v_amd import face
    det = face.RetinaFaceDetection(device=DEV, net=retina)
    img, _ = _retina_input(12, 150, 190)
    maps = det.head_maps(torch.from_numpy(img).to(DEV))
    from s2v_amd.models import retina_outputs
    loc, conf, lms = (t[0].cpu() for t in retina_outputs(face._ctx(DEV), maps, 150, 190))
    thr = _threshold(conf, 0.03)                                 # synthetic weights: a few % of anchors pass
    dets, lmk = det.detect(img, confidence_threshold=thr)
    rd, rl = OF.postprocess(loc, conf, lms, 150, 190, confidence_threshold=thr)
    assert len(dets) == len(rd) and len(dets) > 0
    np.testing.assert_allclose(dets, rd, rtol=3e-7, atol=1e-4)
    np.testing.assert_allclose(lmk, rl, rtol=3e-7, atol=1e-4)


def test_retinaface_detect_large_frame_branch(retina):
    """Frames over 1500 px are resized by 1000 / max side first (retinaface_detection.py:66-70)."""
    from s2v_amd import face
    det = face.RetinaFaceDetection(device=DEV, net=retina)
    img = rng_u8(13, (1520, 760, 3))
    ss = 1000.0 / 1520
    small = OP.resize_linear(np.float32(img), (int(round(760 * ss)), int(round(1520 * ss))), fxfy=(ss, ss))
    maps = det.head_maps(torch.from_numpy(small).to(DEV))
    from s2v_amd.models import retina_outputs
    loc, conf, lms = (t[0].cpu() for t in retina_outputs(face._ctx(DEV), maps, *small.shape[:2]))
    thr = _threshold(conf, 0.005)
    dets, lmk = det.detect(img, confidence_threshold=thr)
    rd, rl = OF.postprocess(loc, conf, lms, *small.shape[:2], ss=ss, confidence_threshold=thr)
    assert len(dets) == len(rd)
    np.testing.assert_allclose(dets, rd, rtol=1e-6, atol=1e-3)


# ----------------------------------------------------------------------------- FaceEnhancement
class _FixedDetector:
    """Detections for the composition tests (the detector itself is tested above)."""

    def __init__(self, dets, landms):
        self.dets, self.landms = np.asarray(dets, np.float32), np.asarray(landms, np.float32)

    def detect(self, img):
        return self.dets, self.landms


def _faces(scale):
    # two faces: a large one and a small one (< 100 px: the filter2D branch), overlapping; one below
    # the 0.9 threshold that must be skipped
    d = np.array([[60, 50, 200, 210, 0.99], [150, 120, 230, 190, 0.95], [10, 10, 40, 40, 0.5]], np.float32) * \
        np.array([scale] * 4 + [1], np.float32)
    lm = np.array([[100, 160, 130, 105, 155, 100, 98, 135, 170, 168],
                   [170, 205, 188, 172, 200, 140, 141, 158, 175, 176],
                   [15, 30, 22, 16, 29, 18, 18, 25, 33, 33]], np.float32) * scale
    return d, lm


@pytest.fixture(scope="module")
def enhancer_nets():
    from s2v_amd import face, models, post, sr
    gpen = models.FullGenerator(512, 512, 8, 2)
    gpen.load_state_dict(synth_sd("gpen"), strict=True)
    parse = models.ParseNet(**models.parse_arch.face_parse_net(512))
    parse.load_state_dict(parsenet_sd(512), strict=True)
    srnet = models.RRDBNet(3, 3, scale=2, num_feat=32, num_block=23, num_grow_ch=32)
    srnet.load_state_dict(rrdb_sd(2), strict=True)
    return dict(facegan=face.FaceGAN(in_size=512, device=DEV, net=gpen.eval()),
                faceparser=post.FaceParse(device=DEV, net=parse.eval()),
                srmodel=sr.RealESRNet(scale=2, device=DEV, net=srnet.eval()))


def _oracle_run(enh, img, ori, trace, of_dev, ef_dev, **kw):
    masks = iter([m.cpu().numpy() for m in trace["masks"]])
    efs = iter([e.cpu().numpy() for e in ef_dev])
    img_sr = None if trace["img_sr"] is None else trace["img_sr"].cpu().numpy()
    out, of, ef = OF.enhance_process(img, ori, detect=lambda im: (trace["dets"], trace["landms"]),
                                     facegan=lambda f: next(efs), parse=lambda f: next(masks),
                                     sr=lambda im: img_sr, use_sr=enh.use_sr, in_size=enh.in_size,
                                     blend=OP.laplacian_blend, **kw)
    assert len(of) == len(of_dev) == 2
    for a, b in zip(of, of_dev):
        assert np.array_equal(a, b.cpu().numpy())                 # warp_and_crop_face bit-exact
    return out


def test_face_enhancement_sr_path_bit_exact(enhancer_nets):
    """The CLI's enhancer (use_sr=True: SR x2, detect on the resized frame, GPEN, paste, blend with
    the SR frame; inference.py:228-231, :319) at in_size 512 (the 2048 crop runs the same kernels)."""
    from s2v_amd import face
    d, lm = _faces(2.0)
    enh = face.FaceEnhancement(in_size=512, use_sr=True, sr_scale=2, device=DEV,
                               facedetector=_FixedDetector(d, lm), **enhancer_nets)
    pp = rng_u8(21, (140, 130, 3))
    ori = rng_u8(22, (280, 260, 3))
    trace = {}
    out, of_dev, ef_dev = enh.process_device(torch.from_numpy(pp).to(DEV), torch.from_numpy(ori).to(DEV),
                                             face_enhance=True, possion_blending=True, trace=trace)
    exp = _oracle_run(enh, pp, ori, trace, of_dev, ef_dev, face_enhance=True, possion_blending=True)
    got = out.cpu().numpy()
    assert got.shape == exp.shape == (280, 260, 3)
    assert np.array_equal(got, exp), int((got != exp).sum())


@pytest.mark.parametrize("possion", [False, True])
def test_face_enhancement_plain_path_bit_exact(enhancer_nets, possion):
    """The reference-frame enhancer (use_sr=False, face_enhance=False: inference.py:225-237) and the
    Laplacian branch with a bbox (face_enhancement.py:176-187)."""
    from s2v_amd import face
    d, lm = _faces(1.0)
    kw = {k: v for k, v in enhancer_nets.items() if k != "srmodel"}
    enh = face.FaceEnhancement(in_size=512, use_sr=False, device=DEV, facedetector=_FixedDetector(d, lm), **kw)
    img = rng_u8(23, (256, 256, 3))
    trace = {}
    bbox = (40, 220, 30, 200) if possion else None
    out, of_dev, ef_dev = enh.process_device(torch.from_numpy(img).to(DEV), torch.from_numpy(img).to(DEV),
                                             face_enhance=not possion, bbox=bbox, possion_blending=possion,
                                             trace=trace)
    exp = _oracle_run(enh, img, img, trace, of_dev, ef_dev, face_enhance=not possion, bbox=bbox,
                      possion_blending=possion)
    got = out.cpu().numpy()
    assert np.array_equal(got, exp), int((got != exp).sum())


def test_face_enhancement_without_faces_fails_like_the_reference(enhancer_nets):
    from s2v_amd import face
    kw = {k: v for k, v in enhancer_nets.items() if k != "srmodel"}
    enh = face.FaceEnhancement(in_size=512, use_sr=False, device=DEV,
                               facedetector=_FixedDetector(np.zeros((0, 5)), np.zeros((0, 10))), **kw)
    img = rng_u8(24, (64, 64, 3))
    with pytest.raises(UnboundLocalError):
        enh.process(img, img)
