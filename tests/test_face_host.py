"""Face detection / alignment restatement (oracle/face.py) on the CPU.

* Against goldens from the reference's own modules (tests/golden/make_golden.py gen_face):
  the RetinaFace FPN + SSH + heads forward (net.py:40-100, retinaface.py:108-125) on synthetic
  backbone features, RetinaFaceDetection.detect's post-processing (retinaface_detection.py:58-124:
  PriorBox, decode, decode_landm, threshold, sort, py_cpu_nms) on synthetic head outputs, and
  get_reference_facial_points / warp_and_crop_face's similarity transforms (align_faces.py).
* The OpenCV restatements (warpAffine, GaussianBlur, getGaussianKernel) have no reference output
  to pin them (OpenCV is absent): parity UNPINNED; here they are checked for the properties
  OpenCV's documented arithmetic guarantees (identity / integer-shift warps are copies, fixed-point
  weights sum to 2^15, normalised symmetric kernels, constant images stay constant).
"""
import numpy as np
import torch

from helpers import FACE_IMG_HW, FACE_LANDMARKS, retina_head_outputs, retina_tail_inputs, synth_sd
from oracle import face


def test_retina_tail_matches_reference(golden):
    g = golden("face_goldens")
    sd = synth_sd("retinaface")
    feats = [torch.from_numpy(f) for f in retina_tail_inputs()]
    with torch.no_grad():
        f = face.fpn(sd, feats)
        loc, conf, landms = face.heads(sd, [face.ssh(sd, f"ssh{i + 1}.", f[i]) for i in range(3)])
    for name, t in (("loc", loc), ("conf", conf), ("landms", landms)):
        ref = g[f"tail_{name}"]
        assert t.shape == ref.shape
        assert np.abs(t.numpy() - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), name


def test_detect_postprocess_matches_reference(golden):
    g = golden("face_goldens")
    loc, conf, lm = retina_head_outputs()
    dets, lms = face.postprocess(torch.from_numpy(loc), torch.from_numpy(conf), torch.from_numpy(lm), *FACE_IMG_HW)
    assert dets.shape == g["det_dets"].shape and len(dets) > 10
    assert np.array_equal(dets, g["det_dets"]) and np.array_equal(lms.astype(np.float32), g["det_landms"])


def test_prior_box_layout():
    pr = face.prior_box(FACE_IMG_HW).numpy()
    h, w = FACE_IMG_HW
    n = sum(2 * (-(-h // s)) * (-(-w // s)) for s in (8, 16, 32))
    assert pr.shape == (n, 4)
    assert np.allclose(pr[0], [4 / w, 4 / h, 16 / w, 16 / h]) and np.allclose(pr[1, 2:], [32 / w, 32 / h])


def test_alignment_matches_reference(golden):
    g = golden("face_goldens")
    for size in (512, 2048):
        ref5 = face.get_reference_facial_points((size, size))
        assert np.array_equal(ref5, g[f"ref5_{size}"])
        for i, pts in enumerate(FACE_LANDMARKS):
            tfm, tfm_inv = face.similarity_transforms(np.array(pts), ref5)
            assert np.array_equal(tfm, g[f"tfm_{i}_{size}"]), (i, size)
            assert np.array_equal(tfm_inv, g[f"tfm_inv_{i}_{size}"]), (i, size)
            # the two transforms are inverse similarities up to fp32 landmark rounding
            A = np.vstack([tfm, [0, 0, 1]]) @ np.vstack([tfm_inv, [0, 0, 1]])
            assert np.abs(A - np.eye(3)).max() < 1e-4 * size


def test_warp_affine_fixed_point_properties():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    assert np.array_equal(face.warp_affine(img, np.array([[1.0, 0, 0], [0, 1.0, 0]]), (53, 37)), img)
    sh = face.warp_affine(img, np.array([[1.0, 0, 5], [0, 1.0, -3]]), (53, 37))
    assert np.array_equal(sh[:34, 5:], img[3:, :48]) and (sh[:, :5] == 0).all() and (sh[34:] == 0).all()
    wf, wi = face._lin_tab()
    assert (wi.sum(1) == 32768).all() and np.allclose(wf.sum(1), 1.0)
    # half-pixel shift: every output is the rounded mean of two neighbours
    hp = face.warp_affine(img, np.array([[1.0, 0, -0.5], [0, 1.0, 0]]), (52, 37))
    exp = (img[:, :52].astype(np.int64) * 16384 + img[:, 1:53].astype(np.int64) * 16384 + 16384) >> 15
    assert np.array_equal(hp, exp.astype(np.uint8))
    # float images: a constant stays constant inside, the border value outside
    f = np.full((20, 30), 0.75, np.float32)
    M = np.array([[0.9, 0.2, 1.3], [-0.2, 0.9, 2.1]])
    out = face.warp_affine(f, M, (30, 20))
    sx, sy, _ = face.warp_coords(M, (30, 20))
    inside = (sx >= 0) & (sx < 29) & (sy >= 0) & (sy < 19)
    assert np.allclose(out[inside], 0.75, atol=1e-7) and out.dtype == np.float32
    assert face.warp_affine(f.astype(np.float64), M, (30, 20)).dtype == np.float64


def test_gaussian_kernel_and_blur():
    for n, s in ((101, 11.0), (9, 1.0)):
        k = face.gaussian_kernel(n, s, np.float64)
        assert abs(k.sum() - 1.0) < 1e-12 and np.array_equal(k, k[::-1]) and k.argmax() == n // 2
    assert len(face.gaussian_kernel(0, 1.0)) == 9
    img = np.full((40, 33), 0.5)
    assert np.allclose(face.gaussian_blur(img, 101, 11), 0.5, atol=1e-12)   # reflect-101 borders
    m = np.zeros((256, 256), np.uint8)
    m[90:170, 80:180] = 255
    m[:10] = 255                                  # inside the zeroed 26-pixel border
    pm = face.mask_postprocess(m / 255.)
    assert pm.dtype == np.float32 and 0.5 < pm.max() < 1 and abs(pm.sum() - 80 * 100) < 80 * 100 * 0.02


def test_convert_scale_abs_rounding():
    x = np.array([-3.5, -0.5, 0.5, 1.5, 2.5, 254.5, 300.0], np.float32)
    assert face.convert_scale_abs(x).tolist() == [4, 0, 0, 2, 2, 254, 255]


# ----------------------------------------------------------------------------- product host logic
def test_product_alignment_and_nms_match_reference(golden):
    from s2v_amd import face as pface
    g = golden("face_goldens")
    for size in (512, 2048):
        ref5 = pface.get_reference_facial_points((size, size), 0.25, (0, 0), True)
        assert np.array_equal(ref5, g[f"ref5_{size}"])
        for i, pts in enumerate(FACE_LANDMARKS):
            tfm, tfm_inv = pface.similarity_transforms(np.array(pts), ref5)
            assert np.array_equal(tfm, g[f"tfm_{i}_{size}"]) and np.array_equal(tfm_inv, g[f"tfm_inv_{i}_{size}"])
    # the device hands over the thresholded candidates in prior order: same NMS result
    loc, conf, lm = retina_head_outputs()
    pr = face.prior_box(FACE_IMG_HW)
    h, w = FACE_IMG_HW
    boxes = (face.decode(torch.from_numpy(loc), pr, face.CFG["variance"]) * torch.Tensor([w, h, w, h])).numpy()
    lms = (face.decode_landm(torch.from_numpy(lm), pr, face.CFG["variance"]) * torch.Tensor([w, h] * 5)).numpy()
    keep = np.where(conf[:, 1] > 0.9)[0]
    dets, lmk = pface.nms_postprocess(boxes[keep], conf[keep, 1], lms[keep])
    assert np.array_equal(dets, g["det_dets"]) and np.array_equal(lmk, g["det_landms"])


def test_paste_window_bounds_the_warped_crop():
    from s2v_amd import face as pface
    rng = np.random.default_rng(1)
    for S, (H, W), pts in ((64, (90, 120), [[30, 52, 41, 33, 50], [40, 41, 52, 63, 62]]),
                           (32, (200, 180), [[20, 150, 90, 30, 140], [30, 35, 100, 160, 170]])):
        ref5 = pface.get_reference_facial_points((S, S), 0.25, (0, 0), True)
        _, tfm_inv = pface.similarity_transforms(np.array(pts, np.float64), ref5)
        mask = rng.random((S, S)).astype(np.float32) + 0.01
        warped = face.warp_affine(mask, tfm_inv, (W, H))
        y0, x0, wh, ww = pface.paste_window(tfm_inv, S, H, W)
        outside = np.ones((H, W), bool)
        outside[y0:y0 + wh, x0:x0 + ww] = False
        assert (warped[outside] == 0).all() and (warped[~outside] > 0).any()


def test_face_entry_points_reject_bad_arguments():
    from s2v_amd import _lib
    lib = _lib.load()
    img = np.zeros((8, 8, 3), np.uint8)
    out = np.zeros((8, 8, 3), np.uint8)
    M = np.zeros(6)
    p = lambda a: a.ctypes.data  # noqa: E731
    assert lib.s2v_warp_affine(p(img), 1, 8, 8, 3, 24, 192, 3, p(M), p(out), 8, 8, 24, 192, None) == -1
    assert lib.s2v_warp_affine(p(img), 1, 8, 8, 3, 8, 192, 0, p(M), p(out), 8, 8, 24, 192, None) == -1
    heads = (_lib.ctypes.c_void_p * 3)(p(img), p(img), p(img))
    hs = (_lib.ctypes.c_int * 3)(13, 7, 4)
    ws = (_lib.ctypes.c_int * 3)(15, 8, 5)                     # 120 / 32 -> 4, not 5
    cand = np.zeros(16 * 1000, np.float32)
    cnt = np.zeros(1, np.int32)
    assert lib.s2v_retina_decode(heads, hs, ws, 32, 100, 120, 0.9, p(cand), p(cnt), 1000, None) == -1
    assert b"level 2" in lib.s2v_last_error()
    assert lib.s2v_gaussian_blur(p(img), 0, 8, 8, 0, p(M), 4, p(out), 1, 2, p(out), 1 << 20, None) == -1   # even ksize
    assert lib.s2v_maxpool2d_nhwc(p(cand), 1, 8, 8, 6, 3, 2, 1, p(cand), 4, 4, None) == -1                 # c % 4


def test_mask_postprocess_mutates_mask_sharp_in_place():
    """face_enhancement.py:83-85: mask[:thres] = 0 ... act on the caller's mask_sharp array, which
    the reference then resizes and warps (:144-150); the restatement must do the same."""
    ms = np.ones((80, 80))
    out = face.mask_postprocess(ms, thres=26)
    assert out.dtype == np.float32
    assert ms[:26].max() == 0 and ms[-26:].max() == 0 and ms[:, :26].max() == 0 and ms[:, -26:].max() == 0
    assert ms[26:-26, 26:-26].min() == 1.0
