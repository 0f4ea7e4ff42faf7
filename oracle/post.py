"""CPU restatement of the mouth-region post-process (TEST INFRASTRUCTURE ONLY; see oracle/__init__).

inference.py:302-313 after ENet + GFPGAN: FaceParse on the restored mouth box, the binary mouth mask
pasted into the frame, three cv2.resize calls to 512x512, Laplacian_Pyramid_Blending_with_mask
(futils/inference_utils.py:181-222) with 10 levels, np.clip and the resize back.

OpenCV is not importable in this image, so cv2.pyrDown / cv2.pyrUp / cv2.resize
(INTER_LINEAR) are restated from OpenCV's imgproc formulas (pyramids.cpp, resize.cpp) with
BORDER_DEFAULT = reflect-101.  PARITY UNPINNED against cv2 itself: the integer paths (uint8 pyrDown,
the fixed-point uint8 resize) follow OpenCV's arithmetic exactly as documented; the float paths use
OpenCV's scalar evaluation order, and a SIMD build of OpenCV may round a few float results
differently (last-bit level, before the final uint8 conversion).  Known-answer tests:
tests/test_post_host.py.  The GPU kernels (csrc/post.hip) evaluate the same expressions and are
compared with this module bit for bit.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def bi101(p, n):
    """cv::borderInterpolate(p, n, BORDER_REFLECT_101), vectorised, any offset."""
    p = np.asarray(p, dtype=np.int64).copy()
    if n == 1:
        return np.zeros_like(p)
    while True:
        bad = (p < 0) | (p >= n)
        if not bad.any():
            return p
        p = np.where(p < 0, -p, np.where(p >= n, 2 * n - 2 - p, p))


def _taps(n_out, n_in):
    o = np.arange(n_out)
    return [bi101(2 * o + d - 2, n_in) for d in range(5)]


def pyr_down(img):
    """cv2.pyrDown (pyramids.cpp pyrDown_): 5x5 [1 4 6 4 1]^2 / 256, output ((h+1)//2, (w+1)//2).
    uint8: integer sum, (s + 128) >> 8; float32: row pass then column pass, x 1/256."""
    h, w = img.shape[:2]
    oh, ow = (h + 1) // 2, (w + 1) // 2
    ty, tx = _taps(oh, h), _taps(ow, w)
    if img.dtype == np.uint8:
        x = img.astype(np.int64)
        c = [x[:, tx[d]] for d in range(5)]
        row = c[2] * 6 + (c[1] + c[3]) * 4 + c[0] + c[4]
        r = [row[ty[d]] for d in range(5)]
        v = r[2] * 6 + (r[1] + r[3]) * 4 + r[0] + r[4]
        return np.clip((v + 128) >> 8, 0, 255).astype(np.uint8)
    x = img.astype(F32)
    c = [x[:, tx[d]] for d in range(5)]
    row = ((c[2] * F32(6) + (c[1] + c[3]) * F32(4)) + c[0]) + c[4]
    r = [row[ty[d]] for d in range(5)]
    v = ((r[2] * F32(6) + (r[1] + r[3]) * F32(4)) + r[0]) + r[4]
    return (v * F32(1.0 / 256)).astype(F32)


def _up_cols(x):
    """Horizontal pass of cv2.pyrUp: [h, w, ...] -> [h, 2w, ...] with OpenCV's edge forms."""
    h, w = x.shape[:2]
    out = np.empty((h, 2 * w) + x.shape[2:], F32)
    if w == 1:
        out[:, 0] = out[:, 1] = x[:, 0] * F32(8)
        return out
    out[:, 0] = x[:, 0] * F32(6) + x[:, 1] * F32(2)
    out[:, 2:2 * w - 2:2] = (x[:, 0:w - 2] + x[:, 1:w - 1] * F32(6)) + x[:, 2:w]
    out[:, 2 * w - 2] = x[:, w - 2] + x[:, w - 1] * F32(7)
    out[:, 1:2 * w - 2:2] = (x[:, 0:w - 1] + x[:, 1:w]) * F32(4)
    out[:, 2 * w - 1] = x[:, w - 1] * F32(8)
    return out


def pyr_up(img):
    """cv2.pyrUp (pyramids.cpp pyrUp_) of a float32 image: output (2h, 2w); source rows for the
    vertical pass are borderInterpolate(2 sy, 2h) / 2; even (R0 + R1*6) + R2, odd (R1 + R2)*4, /64."""
    x = img.astype(F32)
    h = x.shape[0]
    R = _up_cols(x)
    Y = np.arange(2 * h)
    y = Y >> 1
    r0, r1, r2 = (bi101(2 * y - 2, 2 * h) >> 1), (bi101(2 * y, 2 * h) >> 1), (bi101(2 * y + 2, 2 * h) >> 1)
    even = ((R[r0] + R[r1] * F32(6)) + R[r2]) * F32(1.0 / 64)
    odd = ((R[r1] + R[r2]) * F32(4)) * F32(1.0 / 64)
    sel = ((Y & 1) == 0).reshape((-1,) + (1,) * (x.ndim - 1))
    return np.where(sel, even, odd).astype(F32)


def laplacian_blend(A, B, m, num_levels=6):
    """Laplacian_Pyramid_Blending_with_mask (futils/inference_utils.py:181-222), same statement order."""
    GA, GB, GM = A.copy(), B.copy(), m.copy()
    gpA, gpB, gpM = [GA], [GB], [GM]
    for _ in range(num_levels):
        GA, GB, GM = pyr_down(GA), pyr_down(GB), pyr_down(GM)
        gpA.append(np.float32(GA))
        gpB.append(np.float32(GB))
        gpM.append(np.float32(GM))
    lpA, lpB, gpMr = [gpA[num_levels - 1]], [gpB[num_levels - 1]], [gpM[num_levels - 1]]
    for i in range(num_levels - 1, 0, -1):
        lpA.append(np.subtract(gpA[i - 1], pyr_up(gpA[i])))
        lpB.append(np.subtract(gpB[i - 1], pyr_up(gpB[i])))
        gpMr.append(gpM[i - 1])
    LS = []
    for la, lb, gm in zip(lpA, lpB, gpMr):
        gm = gm[:, :, np.newaxis]
        LS.append(la * gm + lb * (1.0 - gm))
    ls_ = LS[0]
    for i in range(1, num_levels):
        ls_ = pyr_up(ls_)
        ls_ = ls_ + LS[i]          # cv2.add of two float32 images
    return ls_.astype(F32)


def _coords(n_out, n_in, clamp, inv_scale=None):
    scale = 1.0 / (n_out / n_in) if inv_scale is None else 1.0 / inv_scale
    f = ((np.arange(n_out) + 0.5) * scale - 0.5).astype(F32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(F32)).astype(F32)
    if clamp:
        lo = s < 0
        f[lo], s[lo] = 0, 0
        hi = s >= n_in - 1
        f[hi], s[hi] = 0, n_in - 1
    return np.clip(s, 0, n_in - 1), np.clip(s + 1, 0, n_in - 1), f


def resize_linear(img, dsize, fxfy=None):
    """cv2.resize(img, dsize=(W, H)) with INTER_LINEAR (resize.cpp resizeGeneric_): uint8 with the
    11-bit fixed-point weights and OpenCV's vector column pass, float32 in float arithmetic, float64
    in double arithmetic with the float coefficients.  ``fxfy``: cv2.resize(img, (0, 0), fx, fy)
    (dsize = the rounded product; the factors themselves scale the coordinates)."""
    W, H = dsize
    h, w = img.shape[:2]
    x0, x1, fx = _coords(W, w, True, None if fxfy is None else fxfy[0])
    y0, y1, fy = _coords(H, h, False, None if fxfy is None else fxfy[1])
    ex = (1,) * (img.ndim - 2)
    if img.dtype == np.uint8:
        a0 = np.rint((F32(1) - fx) * F32(2048)).astype(np.int64).reshape((1, W) + ex)
        a1 = np.rint(fx * F32(2048)).astype(np.int64).reshape((1, W) + ex)
        b0 = np.rint((F32(1) - fy) * F32(2048)).astype(np.int64).reshape((H, 1) + ex)
        b1 = np.rint(fy * F32(2048)).astype(np.int64).reshape((H, 1) + ex)
        S = img.astype(np.int64)
        D = S[:, x0] * a0 + S[:, x1] * a1
        v = (((D[y0] >> 4) * b0) >> 16) + (((D[y1] >> 4) * b1) >> 16)
        return np.clip((v + 2) >> 2, 0, 255).astype(np.uint8)
    if img.dtype == np.float64:
        a0, a1 = (F32(1) - fx).astype(np.float64).reshape((1, W) + ex), fx.astype(np.float64).reshape((1, W) + ex)
        b0, b1 = (F32(1) - fy).astype(np.float64).reshape((H, 1) + ex), fy.astype(np.float64).reshape((H, 1) + ex)
        D = img[:, x0] * a0 + img[:, x1] * a1
        return D[y0] * b0 + D[y1] * b1
    S = img.astype(F32)
    a0, a1 = (F32(1) - fx).reshape((1, W) + ex), fx.reshape((1, W) + ex)
    b0, b1 = (F32(1) - fy).reshape((H, 1) + ex), fy.reshape((H, 1) + ex)
    D = S[:, x0] * a0 + S[:, x1] * a1
    return (D[y0] * b0 + D[y1] * b1).astype(F32)


# ----------------------------------------------------------------------------- FaceParse glue
MASK_COLORMAP = [0] * 10 + [255, 255, 255] + [0] * 6          # face_parsing.py:30
PROCESS_MM = [0] + [255] * 12 + [0] * 6                        # face_parsing.py:39 default
MOUTH_MM = [0] * 10 + [255, 255, 255] + [0] * 6                # inference.py:304


def img2tensor(img):
    """face_parsing.py:59-63: BGR uint8 HWC -> float32 NCHW RGB in [-1, 1] (float64 math)."""
    x = img[..., ::-1] / 255. * 2 - 1
    return np.ascontiguousarray(x.transpose(2, 0, 1)[None]).astype(F32)


def tenor2mask(logits, masks):
    """face_parsing.py:65-81: argmax over channel 1 -> colormap, uint8 [H, W] per image."""
    cls = np.asarray(logits).argmax(axis=1)
    lut = np.asarray(masks, dtype=np.float64)
    return [lut[c].astype(np.uint8) for c in cls]


def mouth_mask_full(tmp_mask, frame_hw, coords):
    """inference.py:305-308: resize the parsing mask to the box, paste resized/255. into a uint8
    frame-sized array (only exact 255 survives, as 1), channel 0 as float32."""
    y1, y2, x1, x2 = coords
    r = resize_linear(tmp_mask, (x2 - x1, y2 - y1))
    full = np.zeros(frame_hw, F32)
    full[y1:y2, x1:x2] = (r == 255).astype(F32)
    return full


def blend_frame(restored, ff, full_mask, levels=10):
    """inference.py:310-313 given the pasted mask: resize to 512, blend, clip, resize back, uint8."""
    height, width = ff.shape[:2]
    A, B, M = (resize_linear(x, (512, 512)) for x in (restored, ff, full_mask))
    img = laplacian_blend(A, B, M, levels)
    return resize_linear(np.clip(img, 0, 255), (width, height)).astype(np.uint8)
