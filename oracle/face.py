"""CPU restatement (test infrastructure only) of GPEN's face detection / alignment / paste-back
 and of FaceEnhancement.process (§8f(2) composition).

Sources restated, each function citing its lines:
  * RetinaFace-R50 forward: third_part/GPEN/face_detect/facemodels/retinaface.py:47-125, net.py:8-100;
    the backbone is torchvision's resnet50 (IntermediateLayerGetter layer2..4), which is ABSENT from
    this image (torchvision is not installed and not vendored) -> backbone parity UNPINNED; the
    FPN / SSH / heads are pinned to the reference modules (tests/golden/make_golden.py imports
    net.py / retinaface.py with empty torchvision import stubs: those classes do not use it).
  * PriorBox (layers/functions/prior_box.py:7-34), decode / decode_landm (utils/box_utils.py:209-247),
    py_cpu_nms (utils/nms/py_cpu_nms.py:10-37), RetinaFaceDetection.detect
    (retinaface_detection.py:58-124): pinned to the reference's own functions (goldens).
  * _umeyama / get_reference_facial_points / warp_and_crop_face (align_faces.py:18-266): the numpy
    parts are pinned (align_faces.py imported with empty cv2 / skimage stubs); cv2.warpAffine,
    GaussianBlur, filter2D, resize and convertScaleAbs are restated from OpenCV's documented
    fixed-point / border semantics -> parity UNPINNED (OpenCV is absent from the image).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

CFG = dict(min_sizes=[[16, 32], [64, 128], [256, 512]], steps=[8, 16, 32], variance=[0.1, 0.2], clip=False)


# ----------------------------------------------------------------------------- network
def _bn(sd, p, x, eps=1e-5):
    return F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"], sd[p + "bias"],
                        False, 0.0, eps)


def _conv_bn(sd, p, x, stride=1, act=None):
    """net.py conv_bn (LeakyReLU(leaky)), conv_bn_no_relu, conv_bn1X1; leaky = 0 at 256 channels."""
    w = sd[p + "0.weight"]
    y = _bn(sd, p + "1.", F.conv2d(x, w, None, stride, w.shape[-1] // 2))
    return F.leaky_relu(y, act) if act is not None else y


def resnet50_body(sd, x, p="body."):
    """torchvision resnet50 conv1..layer4 (Bottleneck v1.5) -> (layer2, layer3, layer4) outputs
    (parameters under prefix ``p``: ``body.`` in RetinaFace, ``backbone.`` in face3d's ReconNet)."""
    y = F.relu(_bn(sd, p + "bn1.", F.conv2d(x, sd[p + "conv1.weight"], None, 2, 3)))
    y = F.max_pool2d(y, 3, 2, 1)
    outs = []
    for li, (planes, blocks, stride) in enumerate(((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))):
        for b in range(blocks):
            q = f"{p}layer{li + 1}.{b}."
            s = stride if b == 0 else 1
            t = F.relu(_bn(sd, q + "bn1.", F.conv2d(y, sd[q + "conv1.weight"])))
            t = F.relu(_bn(sd, q + "bn2.", F.conv2d(t, sd[q + "conv2.weight"], None, s, 1)))
            t = _bn(sd, q + "bn3.", F.conv2d(t, sd[q + "conv3.weight"]))
            idn = _bn(sd, q + "downsample.1.", F.conv2d(y, sd[q + "downsample.0.weight"], None, s)) if b == 0 else y
            y = F.relu(t + idn)
        if li >= 1:
            outs.append(y)
    return outs


def fpn(sd, feats):
    """net.py:79-100."""
    o1 = _conv_bn(sd, "fpn.output1.", feats[0], act=0.0)
    o2 = _conv_bn(sd, "fpn.output2.", feats[1], act=0.0)
    o3 = _conv_bn(sd, "fpn.output3.", feats[2], act=0.0)
    o2 = _conv_bn(sd, "fpn.merge2.", o2 + F.interpolate(o3, size=[o2.size(2), o2.size(3)], mode="nearest"), act=0.0)
    o1 = _conv_bn(sd, "fpn.merge1.", o1 + F.interpolate(o2, size=[o1.size(2), o1.size(3)], mode="nearest"), act=0.0)
    return [o1, o2, o3]


def ssh(sd, p, x):
    """net.py:54-66."""
    c3 = _conv_bn(sd, p + "conv3X3.", x)
    c51 = _conv_bn(sd, p + "conv5X5_1.", x, act=0.0)
    c5 = _conv_bn(sd, p + "conv5X5_2.", c51)
    c72 = _conv_bn(sd, p + "conv7X7_2.", c51, act=0.0)
    c7 = _conv_bn(sd, p + "conv7x7_3.", c72)
    return F.relu(torch.cat([c3, c5, c7], 1))


def heads(sd, features):
    """retinaface.py:108-125 (phase 'test': softmax over the class logits)."""
    def head(name, i, f, k):
        y = F.conv2d(f, sd[f"{name}.{i}.conv1x1.weight"], sd[f"{name}.{i}.conv1x1.bias"])
        return y.permute(0, 2, 3, 1).contiguous().view(y.shape[0], -1, k)
    loc = torch.cat([head("BboxHead", i, f, 4) for i, f in enumerate(features)], 1)
    conf = torch.cat([head("ClassHead", i, f, 2) for i, f in enumerate(features)], 1)
    landm = torch.cat([head("LandmarkHead", i, f, 10) for i, f in enumerate(features)], 1)
    return loc, F.softmax(conf, dim=-1), landm


def retinaface_forward(sd, x):
    """x: [B,3,H,W] float (BGR minus (104,117,123)) -> loc, conf, landms."""
    f = fpn(sd, resnet50_body(sd, x))
    return heads(sd, [ssh(sd, "ssh1.", f[0]), ssh(sd, "ssh2.", f[1]), ssh(sd, "ssh3.", f[2])])


# ----------------------------------------------------------------------------- post-processing
def prior_box(image_size, cfg=CFG):
    """prior_box.py:7-34."""
    anchors = []
    for k, step in enumerate(cfg["steps"]):
        fh, fw = math.ceil(image_size[0] / step), math.ceil(image_size[1] / step)
        for i in range(fh):
            for j in range(fw):
                for ms in cfg["min_sizes"][k]:
                    anchors += [(j + 0.5) * step / image_size[1], (i + 0.5) * step / image_size[0],
                                ms / image_size[1], ms / image_size[0]]
    out = torch.Tensor(anchors).view(-1, 4)
    return out.clamp_(max=1, min=0) if cfg["clip"] else out


def decode(loc, priors, v):
    """box_utils.py:209-227."""
    boxes = torch.cat((priors[:, :2] + loc[:, :2] * v[0] * priors[:, 2:], priors[:, 2:] * torch.exp(loc[:, 2:] * v[1])), 1)
    boxes[:, :2] -= boxes[:, 2:] / 2
    boxes[:, 2:] += boxes[:, :2]
    return boxes


def decode_landm(pre, priors, v):
    """box_utils.py:229-247."""
    return torch.cat([priors[:, :2] + pre[:, 2 * i: 2 * i + 2] * v[0] * priors[:, 2:] for i in range(5)], 1)


def py_cpu_nms(dets, thresh):
    """nms/py_cpu_nms.py:10-37."""
    x1, y1, x2, y2, scores = dets[:, 0], dets[:, 1], dets[:, 2], dets[:, 3], dets[:, 4]
    areas = (x2 - x1 + 1) * (y2 - y1 + 1)
    order = scores.argsort()[::-1]
    keep = []
    while order.size > 0:
        i = order[0]
        keep.append(i)
        xx1 = np.maximum(x1[i], x1[order[1:]])
        yy1 = np.maximum(y1[i], y1[order[1:]])
        xx2 = np.minimum(x2[i], x2[order[1:]])
        yy2 = np.minimum(y2[i], y2[order[1:]])
        w = np.maximum(0.0, xx2 - xx1 + 1)
        h = np.maximum(0.0, yy2 - yy1 + 1)
        inter = w * h
        ovr = inter / (areas[i] + areas[order[1:]] - inter)
        order = order[np.where(ovr <= thresh)[0] + 1]
    return keep


def postprocess(loc, conf, landms, im_height, im_width, ss=1.0, confidence_threshold=0.9, nms_threshold=0.4,
                top_k=5000, keep_top_k=750):
    """retinaface_detection.py:81-124 for one image (loc [P,4], conf [P,2], landms [P,10] tensors)."""
    priors = prior_box((im_height, im_width))
    scale = torch.Tensor([im_width, im_height, im_width, im_height])
    boxes = (decode(loc, priors, CFG["variance"]) * scale).numpy()
    scores = conf.numpy()[:, 1]
    scale1 = torch.Tensor([im_width, im_height] * 5)
    lm = (decode_landm(landms, priors, CFG["variance"]) * scale1).numpy()
    inds = np.where(scores > confidence_threshold)[0]
    boxes, lm, scores = boxes[inds], lm[inds], scores[inds]
    order = scores.argsort()[::-1][:top_k]
    boxes, lm, scores = boxes[order], lm[order], scores[order]
    dets = np.hstack((boxes, scores[:, np.newaxis])).astype(np.float32, copy=False)
    keep = py_cpu_nms(dets, nms_threshold)
    dets, lm = dets[keep, :][:keep_top_k, :], lm[keep][:keep_top_k, :]
    lm = lm.reshape((-1, 5, 2)).transpose((0, 2, 1)).reshape(-1, 10)
    return dets / ss, lm / ss


def detect(sd, img_raw):
    """RetinaFaceDetection.detect (retinaface_detection.py:58-124) on a uint8 HWC BGR frame
    (max side <= 1500: the cv2.resize branch is not taken)."""
    img = np.float32(img_raw)
    h, w = img.shape[:2]
    assert max(h, w) <= 1500, "restatement covers frames up to 1500 px"
    img -= (104, 117, 123)
    x = torch.from_numpy(img.transpose(2, 0, 1).copy()).unsqueeze(0)
    with torch.no_grad():
        loc, conf, landms = retinaface_forward(sd, x)
    return postprocess(loc[0], conf[0], landms[0], h, w)


# ----------------------------------------------------------------------------- alignment
REFERENCE_FACIAL_POINTS = [[30.29459953, 51.69630051], [65.53179932, 51.50139999], [48.02519989, 71.73660278],
                           [33.54930115, 92.3655014], [62.72990036, 92.20410156]]
DEFAULT_CROP_SIZE = (96, 112)


def umeyama(src, dst, estimate_scale=True, scale=1.0):
    """align_faces.py:34-95 (_umeyama)."""
    num, dim = src.shape
    src_mean, dst_mean = src.mean(axis=0), dst.mean(axis=0)
    src_demean, dst_demean = src - src_mean, dst - dst_mean
    A = dst_demean.T @ src_demean / num
    d = np.ones((dim,), dtype=np.double)
    if np.linalg.det(A) < 0:
        d[dim - 1] = -1
    T = np.eye(dim + 1, dtype=np.double)
    U, S, V = np.linalg.svd(A)
    rank = np.linalg.matrix_rank(A)
    if rank == 0:
        return np.nan * T
    elif rank == dim - 1:
        if np.linalg.det(U) * np.linalg.det(V) > 0:
            T[:dim, :dim] = U @ V
        else:
            s = d[dim - 1]
            d[dim - 1] = -1
            T[:dim, :dim] = U @ np.diag(d) @ V
            d[dim - 1] = s
    else:
        T[:dim, :dim] = U @ np.diag(d) @ V
    if estimate_scale:
        scale = 1.0 / src_demean.var(axis=0).sum() * (S @ d)
    T[:dim, dim] = dst_mean - scale * (T[:dim, :dim] @ src_mean.T)
    T[:dim, :dim] *= scale
    return T, scale


def get_reference_facial_points(output_size, inner_padding_factor=0.25, outer_padding=(0, 0), default_square=True):
    """align_faces.py:103-195 on the FaceEnhancement arguments (square crop, inner padding 0.25)."""
    tmp_5pts = np.array(REFERENCE_FACIAL_POINTS)
    tmp_crop_size = np.array(DEFAULT_CROP_SIZE)
    if default_square:
        size_diff = max(tmp_crop_size) - tmp_crop_size
        tmp_5pts += size_diff / 2
        tmp_crop_size += size_diff
    if inner_padding_factor > 0:
        size_diff = tmp_crop_size * inner_padding_factor * 2
        tmp_5pts += size_diff / 2
        tmp_crop_size += np.round(size_diff).astype(np.int32)
    size_bf_outer_pad = np.array(output_size) - np.array(outer_padding) * 2
    scale_factor = size_bf_outer_pad[0].astype(np.float32) / tmp_crop_size[0]
    return tmp_5pts * scale_factor + np.array(outer_padding)


def similarity_transforms(facial_pts, reference_pts):
    """warp_and_crop_face's 'smilarity' branch (align_faces.py:251-258) -> (tfm, tfm_inv) float64 2x3."""
    ref_pts = np.float32(reference_pts)
    if ref_pts.shape[0] == 2:
        ref_pts = ref_pts.T
    src_pts = np.float32(facial_pts)
    if src_pts.shape[0] == 2:
        src_pts = src_pts.T
    params, scale = umeyama(src_pts, ref_pts)
    tfm = params[:2, :]
    params, _ = umeyama(ref_pts, src_pts, False, scale=1.0 / scale)
    return tfm, params[:2, :]


# ----------------------------------------------------------------------------- OpenCV restatements
def invert_affine(M):
    """cv::invertAffineTransform as warpAffine does it without WARP_INVERSE_MAP (double)."""
    M = np.asarray(M, np.float64).reshape(6).copy()
    D = M[0] * M[4] - M[1] * M[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = M[4] * D, M[0] * D
    M[0], M[1], M[3], M[4] = A11, -M[1] * D, -M[3] * D, A22
    b1 = -M[0] * M[2] - M[1] * M[5]
    b2 = -M[3] * M[2] - M[4] * M[5]
    M[2], M[5] = b1, b2
    return M


def _lin_tab():
    """cv::initInterTab2D(INTER_LINEAR): 32x32 fractions (fy, fx) -> tap weights (y0x0, y0x1, y1x0, y1x1)
    as float32 (1-t, t products, exact: multiples of 2^-10) and as the int16 fixed-point weights
    saturate_cast<short>(w * 2^15), which already sum to 2^15 (no rounding correction is needed)."""
    t = np.arange(32, dtype=np.float32) / np.float32(32)
    c = np.stack([1 - t, t], 1)                                  # [32, 2] 1-D coefficients
    wf = (c[:, None, :, None] * c[None, :, None, :]).astype(np.float32).reshape(32 * 32, 4)
    wi = (wf.astype(np.float64) * 32768).astype(np.int64)
    assert (wi.sum(1) == 32768).all() and (wi == wf.astype(np.float64) * 32768).all()
    return wf, wi


_TAB = None


def warp_coords(M, dsize):
    """WarpAffineInvoker's fixed-point source coordinates for dst pixel (x, y): (sx, sy, alpha) with
    AB_BITS = 10 (saturate_cast<int> = round-half-even), round_delta 16, INTER_BITS = 5, sx / sy
    saturated to int16."""
    ow, oh = dsize
    Mi = invert_affine(M)
    x = np.arange(ow, dtype=np.float64)
    adelta = np.rint(Mi[0] * x * 1024).astype(np.int64)
    bdelta = np.rint(Mi[3] * x * 1024).astype(np.int64)
    y = np.arange(oh, dtype=np.float64)
    X0 = np.rint((Mi[1] * y + Mi[2]) * 1024).astype(np.int64) + 16
    Y0 = np.rint((Mi[4] * y + Mi[5]) * 1024).astype(np.int64) + 16
    X = (X0[:, None] + adelta[None, :]) >> 5
    Y = (Y0[:, None] + bdelta[None, :]) >> 5
    sx, sy = np.clip(X >> 5, -32768, 32767), np.clip(Y >> 5, -32768, 32767)
    return sx, sy, (Y & 31) * 32 + (X & 31)


def warp_affine(src, M, dsize, border_value=0):
    """cv2.warpAffine(src, M, dsize, flags=INTER_LINEAR or INTER_AREA (mapped to INTER_LINEAR),
    BORDER_CONSTANT) for uint8 / float32 / float64 images (remapBilinear): uint8 through the 15-bit
    integer weights ((sum + 2^14) >> 15), float through the float weights, summed in tap order
    ((v00 w0 + v01 w1) + v10 w2) + v11 w3 in the image's own precision."""
    global _TAB
    if _TAB is None:
        _TAB = _lin_tab()
    wf, wi = _TAB
    src = np.asarray(src)
    h, w = src.shape[:2]
    squeeze = src.ndim == 2
    s = src[..., None] if squeeze else src
    sx, sy, alpha = warp_coords(M, dsize)
    acc = None
    for k, (dy, dx) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
        yy, xx = sy + dy, sx + dx
        inside = (yy >= 0) & (yy < h) & (xx >= 0) & (xx < w)
        v = np.where(inside[..., None], s[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)], border_value)
        if s.dtype == np.uint8:
            term = v.astype(np.int64) * wi[alpha, k][..., None]
        else:
            term = v.astype(s.dtype) * wf[alpha, k][..., None].astype(s.dtype)
        acc = term if acc is None else acc + term
    if s.dtype == np.uint8:
        r = np.clip((acc + (1 << 14)) >> 15, 0, 255).astype(np.uint8)
    else:
        r = acc.astype(s.dtype)
    return r[..., 0] if squeeze else r


def warp_and_crop_face(src_img, facial_pts, reference_pts, crop_size):
    """align_faces.py:210-266 ('smilarity') -> (face_img, tfm_inv)."""
    tfm, tfm_inv = similarity_transforms(facial_pts, reference_pts)
    return warp_affine(src_img, tfm, (crop_size[0], crop_size[1])), tfm_inv


def gaussian_kernel(ksize, sigma, dtype=np.float32):
    """cv::getGaussianKernel (OpenCV 4.x getGaussianKernelBitExact, restated in IEEE double with
    math.exp for softdouble's exp): t_i = exp((x*x) * (-0.125 / sigma^2)) for x = 1 - n, 3 - n, ..
    over the first half, sum = 2 * sum(t) + 1, k_i = t_i * (1 / sum), centre 1 * (1 / sum); cast to
    the image's kernel type (CV_32F for float32 images, CV_64F for float64).  ksize <= 0: the size
    GaussianBlur derives for float images, cvRound(sigma * 8 + 1) | 1."""
    if ksize <= 0:
        ksize = int(np.rint(sigma * 4 * 2 + 1)) | 1
    n = ksize
    assert n % 2 == 1 and sigma > 0
    scale2x = -0.125 / (sigma * sigma)
    half = (n - 1) // 2
    vals, tot = [], 0.0
    for i in range(half):
        x = 1 - n + 2 * i
        t = math.exp(float(x * x) * scale2x)
        vals.append(t)
        tot += t
    tot = tot * 2.0 + 1.0
    mul = 1.0 / tot
    k = [v * mul for v in vals]
    k = k + [1.0 * mul] + k[::-1]
    return np.array(k, dtype=np.float64).astype(dtype)


def _reflect101(i, n):
    i = np.abs(i)
    return np.where(i >= n, 2 * n - 2 - i, i)


def gaussian_blur(img, ksize, sigma):
    """cv2.GaussianBlur(img, (ksize, ksize), sigma) on a single-channel float32 / float64 image,
    BORDER_REFLECT_101, as sepFilter2D's non-IPP path computes it in the image's precision: the row
    pass sums k[t] * x[t] in tap order (RowFilter), the column pass is SymmColumnFilter:
    k[c] * centre + sum_j k[c + j] * (below_j + above_j).  (OpenCV's AVX2 float32 path contracts
    these into FMAs; this restatement rounds every product, a difference of <= a few ulp.)"""
    a = np.asarray(img)
    dt = a.dtype
    assert dt in (np.float32, np.float64) and a.ndim == 2
    k = gaussian_kernel(ksize, sigma, dt)
    r = len(k) // 2
    h, w = a.shape
    cols = _reflect101(np.arange(w)[:, None] + np.arange(-r, r + 1)[None, :], w)
    tmp = a[:, cols[:, 0]] * k[0]
    for t in range(1, len(k)):
        tmp = tmp + a[:, cols[:, t]] * k[t]
    rows = _reflect101(np.arange(h)[:, None] + np.arange(-r, r + 1)[None, :], h)
    out = tmp * k[r]
    for j in range(1, r + 1):
        out = out + (tmp[rows[:, r + j], :] + tmp[rows[:, r - j], :]) * k[r + j]
    return out.astype(dt)


def mask_postprocess(mask, thres=26):
    """face_enhancement.py:83-88 on mask_sharp = parse / 255. (float64): zero a thres-pixel border
    IN PLACE (the caller's mask_sharp keeps the zeroed border, as the reference's does: :144-150 go
    on to resize and warp that same array), then two 101x101 sigma-11 Gaussian blurs in float64,
    astype float32."""
    if not (isinstance(mask, np.ndarray) and mask.dtype == np.float64):
        mask = np.array(mask, dtype=np.float64)
    mask[:thres, :] = 0
    mask[-thres:, :] = 0
    mask[:, :thres] = 0
    mask[:, -thres:] = 0
    mask = gaussian_blur(mask, 101, 11)
    mask = gaussian_blur(mask, 101, 11)
    return mask.astype(np.float32)


def convert_scale_abs(x):
    """cv2.convertScaleAbs: saturate_cast<uchar>(|x|) with round-half-even."""
    return np.clip(np.rint(np.abs(x)), 0, 255).astype(np.uint8)


# ----------------------------------------------------------------------------- FaceEnhancement
FACE_MM = [0, 255, 255, 255, 255, 255, 255, 255, 0, 0, 255, 255, 255, 0, 0, 0, 0, 0, 0]   # face_enhancement.py:136
SMALL_FACE_KERNEL = np.array([[0.0625, 0.125, 0.0625], [0.125, 0.25, 0.125], [0.0625, 0.125, 0.0625]], np.float32)


def filter2d_u8(img, kern):
    """cv2.filter2D(img, -1, kern 3x3 fp32) on uint8, BORDER_REFLECT_101, fp32 sum in row-major tap
    order, cvRound, saturated."""
    h, w = img.shape[:2]
    ys = _reflect101(np.arange(h)[:, None] + np.arange(-1, 2)[None, :], h)
    xs = _reflect101(np.arange(w)[:, None] + np.arange(-1, 2)[None, :], w)
    s = np.zeros(img.shape, np.float32)
    for dy in range(3):
        for dx in range(3):
            s = s + kern[dy, dx] * img[ys[:, dy]][:, xs[:, dx]].astype(np.float32)
    return np.clip(np.rint(s), 0, 255).astype(np.uint8)


def paste_window(tfm_inv, S, H, W):
    """Frame window holding every pixel whose warped crop value can be non-zero (the image of the
    crop square (-1, S) x (-1, S) under tfm_inv, padded for the fixed-point rounding)."""
    M = np.asarray(tfm_inv, np.float64)
    cs = np.array([[-2.0, -2.0], [S + 1.0, -2.0], [-2.0, S + 1.0], [S + 1.0, S + 1.0]])
    p = cs @ M[:, :2].T + M[:, 2]
    pad = 2.0 + 2.0 * max(1.0, float(np.abs(M[:, :2]).sum(1).max()))
    x0, y0 = int(max(0, np.floor(p[:, 0].min() - pad))), int(max(0, np.floor(p[:, 1].min() - pad)))
    x1, y1 = int(min(W, np.ceil(p[:, 0].max() + pad))), int(min(H, np.ceil(p[:, 1].max() + pad)))
    return y0, x0, max(0, y1 - y0), max(0, x1 - x0)


def enhance_process(img, ori_img, *, detect, facegan, parse, sr, use_sr, in_size, face_enhance=True, bbox=None,
                    possion_blending=False, threshold=0.9, blend=None):
    """FaceEnhancement.process (face_enhancement.py:91-193) with the networks given as callables
    (detect: uint8 frame -> (dets, landms); facegan: uint8 S x S face -> uint8 face; parse: uint8
    face -> uint8 512 x 512 mask with FACE_MM; sr: uint8 frame -> uint8 frame or None) and every
    OpenCV call restated above.  ``blend``: the Laplacian pyramid blend (possion_blending branch).
    Returns (img, orig_faces, enhanced_faces)."""
    from . import post as opost
    orig_faces, enhanced_faces = [], []
    img_sr = None
    if use_sr:
        img_sr = sr(img)
        if img_sr is not None:
            img = opost.resize_linear(img, img_sr.shape[:2][::-1])
    facebs, landms = detect(img)
    height, width = img.shape[:2]
    full_mask = np.zeros((height, width), dtype=np.float32)
    full_img = np.zeros(ori_img.shape, dtype=np.uint8)
    ref5 = get_reference_facial_points((in_size, in_size))
    mask_sharp = None
    for faceb, facial5points in zip(facebs, landms):
        if faceb[4] < threshold:
            continue
        fh, fw = (faceb[3] - faceb[1]), (faceb[2] - faceb[0])
        tfm, tfm_inv = similarity_transforms(np.reshape(facial5points, (2, 5)), ref5)
        of = warp_affine(img, tfm, (in_size, in_size))
        ef = facegan(of) if face_enhance else of
        orig_faces.append(of)
        enhanced_faces.append(ef)
        mask_sharp = parse(ef) / 255.
        tmp_mask = mask_postprocess(mask_sharp)
        tmp_mask = opost.resize_linear(tmp_mask, (in_size, in_size))
        tmp_mask = warp_affine(tmp_mask, tfm_inv, (width, height))
        mask_sharp = opost.resize_linear(mask_sharp, ef.shape[:2])
        mask_sharp = warp_affine(mask_sharp, tfm_inv, (width, height))
        if min(fh, fw) < 100:
            ef = filter2d_u8(ef, SMALL_FACE_KERNEL)
        tmp_img = warp_affine(ef, tfm_inv, (width, height))
        sel = (tmp_mask - full_mask) > 0
        full_mask[sel] = tmp_mask[sel]
        full_img[sel] = tmp_img[sel]
    if mask_sharp is None:
        raise UnboundLocalError("local variable 'mask_sharp' referenced before assignment (no face above the "
                                "threshold: face_enhancement.py:165 fails the same way)")
    mask_sharp = gaussian_blur(mask_sharp, 0, 1.0)
    full_mask = full_mask[:, :, np.newaxis]
    mask_sharp = mask_sharp[:, :, np.newaxis]
    if use_sr and img_sr is not None:
        return convert_scale_abs(img_sr * (1 - full_mask) + full_img * full_mask), orig_faces, enhanced_faces
    if possion_blending:
        if bbox is not None:
            y1, y2, x1, x2 = bbox
            mask_bbox = np.zeros_like(mask_sharp)
            mask_bbox[y1:y2 - 5, x1:x2] = 1
            full_img, ori_img, full_mask = [opost.resize_linear(x, (512, 512)) for x in
                                            (full_img, ori_img, np.float32(mask_sharp * mask_bbox)[..., 0])]
        else:
            full_img, ori_img, full_mask = [opost.resize_linear(x, (512, 512)) for x in
                                            (full_img, ori_img, full_mask[..., 0])]
        out = blend(full_img, ori_img, full_mask, 6)
        out = np.clip(out, 0, 255)
        return opost.resize_linear(out.astype(np.float32), (width, height)).astype(np.uint8), orig_faces, \
            enhanced_faces
    out = convert_scale_abs(ori_img * (1 - full_mask) + full_img * full_mask)
    out = convert_scale_abs_f64(ori_img * (1 - mask_sharp) + out * mask_sharp)
    return out, orig_faces, enhanced_faces


def convert_scale_abs_f64(x):
    """cv2.convertScaleAbs of a float64 image as OpenCV's vector path does it: each value rounded to
    fp32 first, then |.|, round half to even, saturated."""
    return convert_scale_abs(np.asarray(x, np.float64).astype(np.float32))
