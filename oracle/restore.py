"""CPU restatement (test infrastructure only) of GFPGANer's restore composition:
third_part/GFPGAN/gfpgan/utils.py:97-143 (GFPGANer.enhance, called at inference.py:300-301 with
upscale=1, only_center_face=True, paste_back=True) and the facexlib helper it drives.

facexlib is a third-party dependency pinned at 0.2.5 (requirements.txt:5) and NOT vendored in the
reference; OpenCV (cv2) is absent from this image.  The functions below restate facexlib 0.2.5's
published algorithm (facexlib/utils/face_restoration_helper.py: FaceRestoreHelper, get_center_face;
facexlib/detection/retinaface.py: RetinaFace.detect_faces) and the OpenCV calls it makes
(estimateAffinePartial2D with LMEDS, invertAffineTransform, warpAffine, erode, GaussianBlur) from
their documented semantics -> parity UNPINNED: no reference output or fixture covers this path.
The pieces shared with GPEN's FaceEnhancement (warpAffine, the Gaussian kernel, the RetinaFace
decode) come from oracle/face.py.
"""
from __future__ import annotations

import itertools
from fractions import Fraction

import numpy as np

from . import face as OF

# FaceRestoreHelper.__init__: the standard 5 landmarks of FFHQ faces at 512 x 512 (template_3points=False)
FFHQ_TEMPLATE_512 = np.array([[192.98138, 239.94708], [318.90277, 240.1936], [256.63416, 314.01935],
                              [201.26117, 371.41043], [313.08905, 371.15118]])
BORDER_GRAY = (135, 133, 132)          # align_warp_face's borderValue
CONF_THRESHOLD = 0.97                  # get_face_landmarks_5: detect_faces(input_img, 0.97)


# ----------------------------------------------------------------------------- detection post-processing
def detect_faces_post(boxes, scores, landms, nms_threshold=0.4):
    """RetinaFace.detect_faces after the threshold (facexlib detection/retinaface.py): the survivors in
    prior order -> sort by score (argsort()[::-1]), py_cpu_nms, [K, 15] float32 rows
    (x1, y1, x2, y2, score, 5 interleaved landmark x, y)."""
    order = scores.argsort()[::-1]
    boxes, landms, scores = boxes[order], landms[order], scores[order]
    bounding_boxes = np.hstack((boxes, scores[:, np.newaxis])).astype(np.float32, copy=False)
    keep = OF.py_cpu_nms(bounding_boxes, nms_threshold)
    return np.concatenate((bounding_boxes[keep, :], landms[keep]), axis=1)


def get_center_face(det_faces, h=0, w=0, center=None):
    """facexlib face_restoration_helper.get_center_face: the face whose box centre is nearest the
    image centre (first on ties)."""
    center = np.array(center) if center is not None else np.array([w / 2, h / 2])
    dist = [np.linalg.norm(np.array([(f[0] + f[2]) / 2, (f[1] + f[3]) / 2]) - center) for f in det_faces]
    idx = dist.index(min(dist))
    return det_faces[idx], idx


def get_largest_face(det_faces, h, w):
    """facexlib face_restoration_helper.get_largest_face: largest box area, boxes clipped to the image."""
    def get_location(val, length):
        if val < 0:
            return 0
        if val > length:
            return length
        return val
    areas = []
    for f in det_faces:
        left, right = get_location(f[0], w), get_location(f[2], w)
        top, bottom = get_location(f[1], h), get_location(f[3], h)
        areas.append((right - left) * (bottom - top))
    idx = areas.index(max(areas))
    return det_faces[idx], idx


def landmarks_5(bboxes, h, w, only_center_face=False, eye_dist_threshold=None):
    """FaceRestoreHelper.get_face_landmarks_5's selection (template_3points=False, no resize, no
    pad_blur) on detect_faces' rows -> (det_faces, all_landmarks_5)."""
    det_faces, lms = [], []
    for bbox in bboxes:
        # facexlib 0.2.5's expression as published, index quirk included (bbox[5:7] / [7:9] are the eyes;
        # it differences [6]-[8] and [7]-[9]); facexlib is not vendored, so this is restated, parity unpinned
        eye_dist = np.linalg.norm([bbox[6] - bbox[8], bbox[7] - bbox[9]])
        if eye_dist_threshold is not None and eye_dist < eye_dist_threshold:
            continue
        lms.append(np.array([[bbox[i], bbox[i + 1]] for i in range(5, 15, 2)]))
        det_faces.append(bbox[0:5])
    if not det_faces:
        return [], []
    if only_center_face:
        det, idx = get_center_face(det_faces, h, w)
        return [det], [lms[idx]]
    return det_faces, lms


# ----------------------------------------------------------------------------- estimateAffinePartial2D
def _partial_from_pair(f, t):
    """AffinePartial2DEstimatorCallback::runKernel: the 4-DOF similarity through two point pairs,
    analytically in double from float32 points."""
    x1, y1, x2, y2 = (float(v) for v in (f[0, 0], f[0, 1], f[1, 0], f[1, 1]))
    X1, Y1, X2, Y2 = (float(v) for v in (t[0, 0], t[0, 1], t[1, 0], t[1, 1]))
    d = 1.0 / ((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2))
    S0 = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2))
    S1 = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2))
    S2 = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) - (X1 * x2 - X2 * x1) * (x1 - x2))
    S3 = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) - (Y1 * y2 - Y2 * y1) * (y1 - y2))
    return np.array([[S0, -S1, S2], [S1, S0, S3]])


def _errors(M, f, t):
    """Affine2DEstimatorCallback::computeError: squared reprojection error per point (double, stored
    as float32)."""
    ff, tt = f.astype(np.float64), t.astype(np.float64)
    a = M[0, 0] * ff[:, 0] + M[0, 1] * ff[:, 1] + M[0, 2] - tt[:, 0]
    b = M[1, 0] * ff[:, 0] + M[1, 1] * ff[:, 1] + M[1, 2] - tt[:, 1]
    return (a * a + b * b).astype(np.float32)


def _ls_partial(f, t):
    """The least-squares 4-DOF similarity over the given pairs: the point the Levenberg-Marquardt
    refinement of estimateAffinePartial2D converges to (its residuals are linear in (a, b, tx, ty))."""
    f, t = f.astype(np.float64), t.astype(np.float64)
    fm, tm = f.mean(0), t.mean(0)
    fd, td = f - fm, t - tm
    den = (fd * fd).sum()
    a = (fd[:, 0] * td[:, 0] + fd[:, 1] * td[:, 1]).sum() / den
    b = (fd[:, 0] * td[:, 1] - fd[:, 1] * td[:, 0]).sum() / den
    tx = tm[0] - (a * fm[0] - b * fm[1])
    ty = tm[1] - (b * fm[0] + a * fm[1])
    return np.array([[a, -b, tx], [b, a, ty]])


def estimate_affine_partial_2d(src, dst):
    """cv2.estimateAffinePartial2D(src, dst, method=cv2.LMEDS)[0] (align_warp_face): both point sets
    as float32; LMeDS over 2-point models, here over EVERY pair of the 5 landmarks (OpenCV draws ~13
    random pairs with a fixed-seed RNG; the exhaustive search returns the model those draws find
    whenever they include the best pair), median = the count / 2-th smallest error; inliers = error
    <= sigma^2 with sigma = max(2.5 * 1.4826 * (1 + 5 / (count - 2)) * sqrt(median), 0.001); then the
    refinement over the inliers (closed-form least squares: the LM optimum).  Returns None when no
    model exists (fewer than 2 points / coincident points)."""
    f, t = np.float32(src).reshape(-1, 2), np.float32(dst).reshape(-1, 2)
    n = len(f)
    if n < 2:
        return None
    best, best_med = None, np.inf
    for i, j in itertools.combinations(range(n), 2):
        if f[i, 0] == f[j, 0] and f[i, 1] == f[j, 1]:
            continue
        M = _partial_from_pair(f[[i, j]], t[[i, j]])
        if n == 2:
            return M
        med = float(np.sort(_errors(M, f, t))[n // 2])
        if med < best_med:
            best, best_med = M, med
    if best is None:
        return None
    sigma = max(2.5 * 1.4826 * (1 + 5.0 / (n - 2)) * np.sqrt(best_med), 0.001)
    inl = _errors(best, f, t) <= np.float32(sigma * sigma)
    if inl.sum() < 2:
        return None
    return _ls_partial(f[inl], t[inl])


def invert_affine_transform(M):
    """cv2.invertAffineTransform (double) -> 2x3."""
    return OF.invert_affine(M).reshape(2, 3)


# ----------------------------------------------------------------------------- paste-back
def erode(img, k):
    """cv2.erode(img, np.ones((k, k), np.uint8)) on a float32 image: anchor (k // 2, k // 2), the
    constant border never wins; an empty kernel (k == 0) is OpenCV's 3 x 3 default."""
    if k == 0:
        k = 3
    h, w = img.shape
    a = k // 2
    pad = np.full((h + k - 1, w + k - 1), np.inf, np.float32)
    pad[a: a + h, a: a + w] = img
    r = np.full((h + k - 1, w), np.inf, np.float32)
    for t in range(k):
        r = np.minimum(r, pad[:, t: t + w])
    out = np.full((h, w), np.inf, np.float32)
    for t in range(k):
        out = np.minimum(out, r[t: t + h])
    return out


def gaussian_taps_auto(k):
    """cv::getGaussianKernel(k, sigma=0, CV_32F) as GaussianBlur(img, (k, k), 0) asks for it (OpenCV
    4.x getGaussianKernelBitExact): the fixed small kernels for k = 1, 3, 5, 7, else sigma =
    k * 0.15 + 0.35 (softdouble mulAdd: one rounding) through oracle.face.gaussian_kernel."""
    fixed = {1: [1.0], 3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
             7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}
    if k in fixed:
        return np.array(fixed[k], np.float32)
    sigma = float(Fraction(k) * Fraction(0.15) + Fraction(0.35))
    return OF.gaussian_kernel(k, sigma, np.float32)


def gaussian_blur_auto(img, k):
    """cv2.GaussianBlur(img, (k, k), 0) on a float32 image: k == 1 copies; else oracle.face's separable
    form (row pass in tap order, SymmColumnFilter column pass, BORDER_REFLECT_101) with the taps above."""
    if k == 1:
        return img.copy()
    taps = gaussian_taps_auto(k)
    r = len(taps) // 2
    h, w = img.shape
    cols = OF._reflect101(np.arange(w)[:, None] + np.arange(-r, r + 1)[None, :], w)
    tmp = img[:, cols[:, 0]] * taps[0]
    for t in range(1, len(taps)):
        tmp = tmp + img[:, cols[:, t]] * taps[t]
    rows = OF._reflect101(np.arange(h)[:, None] + np.arange(-r, r + 1)[None, :], h)
    out = tmp * taps[r]
    for j in range(1, r + 1):
        out = out + (tmp[rows[:, r + j], :] + tmp[rows[:, r - j], :]) * taps[r + j]
    return out.astype(np.float32)


def paste_faces(input_img, restored_faces, inverse_affines, face_size=(512, 512), trace=None):
    """FaceRestoreHelper.paste_faces_to_input_image (upscale_factor 1, upsample_img None, use_parse
    False): the background is the input itself (cv2.resize to the same size copies), then per face
    inv_restored = warpAffine(face, inverse_affine), inv_mask = warpAffine(ones), 2 x 2 erosion,
    pasted_face, total_face_area = np.sum (float32), w_edge = int(area ** 0.5) // 20, a
    (2 w_edge)^2 erosion, GaussianBlur(2 w_edge + 1, sigma 0), the fp32 blend; astype(uint8)."""
    h, w = input_img.shape[:2]
    up = input_img
    for face, inv in zip(restored_faces, inverse_affines):
        inv_restored = OF.warp_affine(face, inv, (w, h))
        inv_mask = OF.warp_affine(np.ones(face_size[::-1], np.float32), inv, (w, h))
        inv_mask_erosion = erode(inv_mask, 2)
        pasted_face = inv_mask_erosion[:, :, None] * inv_restored
        total_face_area = np.sum(inv_mask_erosion)
        w_edge = int(total_face_area ** 0.5) // 20
        inv_mask_center = erode(inv_mask_erosion, w_edge * 2)
        inv_soft_mask = gaussian_blur_auto(inv_mask_center, w_edge * 2 + 1)[:, :, None]
        up = inv_soft_mask * pasted_face + (1 - inv_soft_mask) * up
        if trace is not None:
            trace.append(dict(erosion=inv_mask_erosion, area=total_face_area, w_edge=w_edge, soft=inv_soft_mask[..., 0]))
    return up.astype(np.uint8)


def tensor2img(x):
    """basicsr tensor2img(x [3, H, W] fp32, rgb2bgr=True, min_max=(-1, 1)) -> uint8 HWC BGR."""
    t = np.clip(np.asarray(x, np.float32), -1, 1)
    t = (t - np.float32(-1)) / np.float32(2)
    img = t.transpose(1, 2, 0)[:, :, ::-1]
    return (img * np.float32(255.0)).round().astype(np.uint8)


def img2tensor_norm(face):
    """GFPGANer.enhance's input: img2tensor(face / 255., bgr2rgb=True, float32=True), then
    normalize((0.5,) * 3, (0.5,) * 3) -> fp32 [3, S, S] RGB."""
    t = (face / 255.).astype(np.float32)[:, :, ::-1].transpose(2, 0, 1)
    return (t - np.float32(0.5)) / np.float32(0.5)


def enhance(img, *, detect_faces, gfpgan, has_aligned=False, only_center_face=False, paste_back=True,
            face_size=512, trace=None):
    """GFPGANer.enhance (gfpgan/utils.py:97-143, upscale 1, bg_upsampler None) with the networks as
    callables: detect_faces(img uint8, conf_threshold) -> [K, 15] rows; gfpgan(x fp32 [3, S, S]) ->
    output fp32 [3, S, S].  Returns (cropped_faces, restored_faces, restored_img or None)."""
    if has_aligned:
        from . import post as opost
        cropped = [opost.resize_linear(img, (face_size, face_size))]
        affines = []
    else:
        h, w = img.shape[:2]
        bboxes = detect_faces(img, CONF_THRESHOLD)
        _, lms = landmarks_5(bboxes, h, w, only_center_face=only_center_face, eye_dist_threshold=5)
        template = FFHQ_TEMPLATE_512 * (face_size / 512.0)
        affines = [estimate_affine_partial_2d(lm, template) for lm in lms]
        cropped = [OF.warp_affine(img, M, (face_size, face_size), border_value=np.array(BORDER_GRAY))
                   for M in affines]
    restored = [tensor2img(gfpgan(img2tensor_norm(f))) for f in cropped]
    if trace is not None:
        trace.update(affines=affines, cropped=cropped, restored=restored, paste=[])
    if has_aligned or not paste_back:
        return cropped, restored, None
    inv = [invert_affine_transform(M) for M in affines]
    out = paste_faces(img, restored, inv, (face_size, face_size), None if trace is None else trace["paste"])
    return cropped, restored, out
