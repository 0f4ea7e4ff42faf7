"""CPU restatement (test infrastructure only) of the 3DMM coefficient extraction that feeds DNet
(SURVEY.md §8f(4)).  Never imported by the product path.

Sources restated, each function citing its lines:
  * Pillow's Image.resize (libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc,
    ImagingResampleHorizontal_8bpc / Vertical_8bpc; bicubic a = -0.5, bilinear) and Image.crop's
    zero fill -> ``pil_resize`` / ``pil_resize_crop``.  Pinned bit-exact against Pillow itself
    (installed in the build image) and against the reference's own resize_n_crop_img
    (tests/golden/face3d_goldens.npz, tests/golden/make_golden.py gen_face3d).
  * third_part/face3d/util/preprocess.py:18-43 POS, :147-167 resize_n_crop_img, :173-179 extract_5p,
    :186-216 align_img; util/load_mats.py:105-116 load_lm3d (5-point reduction) -> pinned to the
    reference functions (goldens).
  * models/networks.py:66-105 ReconNetWrapper('resnet50', use_last_fc=False), :226-372 ResNet ->
    ``recon_forward``; pinned to the reference module's output on synthetic weights (goldens).
  * preprocessing/facing.py:108-129 (the per-frame landmark fix-up, the /255 input, split_coeff
    futils/inference_utils.py:158-181 and the 262-float semantic row) -> ``face_3dmm_extraction``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .face import resnet50_body, _bn  # noqa: F401

PREC = 22


# ----------------------------------------------------------------------------- Pillow resample
def _filter(kind, x):
    x = np.abs(x)
    if kind == 3:                                   # bicubic_filter, a = -0.5
        a = -0.5
        return np.where(x < 1.0, ((a + 2.0) * x - (a + 3.0)) * x * x + 1,
                        np.where(x < 2.0, (((x - 5) * x + 8) * x - 4) * a, 0.0))
    return np.where(x < 1.0, 1.0 - x, 0.0)           # bilinear_filter


def pil_coeffs(in_size, out_size, kind=3):
    """precompute_coeffs + normalize_coeffs_8bpc -> dense int64 matrix [out_size, in_size]."""
    support0 = 2.0 if kind == 3 else 1.0
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = support0 * filterscale
    ss = 1.0 / filterscale
    K = np.zeros((out_size, in_size), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = _filter(kind, (np.arange(xmax) + xmin - center + 0.5) * ss)
        ww = 0.0
        for v in w:                                  # running sum in tap order
            ww += float(v)
        if ww != 0.0:
            w = w / ww
        K[xx, xmin:xmin + xmax] = np.where(w < 0, (-0.5 + w * (1 << PREC)).astype(np.int64),
                                           (0.5 + w * (1 << PREC)).astype(np.int64))
    return K


def _clip8(acc):
    return np.clip(acc >> PREC, 0, 255).astype(np.uint8)


def pil_resize(img, w, h, kind=3):
    """Image.resize((w, h), kind) of a uint8 HWC RGB array: horizontal pass (uint8 rows) then
    vertical; a pass whose size does not change is skipped (ImagingResampleInner)."""
    h0, w0 = img.shape[:2]
    x = img.astype(np.int64)
    if w != w0:
        K = pil_coeffs(w0, w, kind)
        x = _clip8(np.einsum("hwc,vw->hvc", x, K) + (1 << (PREC - 1))).astype(np.int64)
    if h != h0:
        K = pil_coeffs(h0, h, kind)
        x = _clip8(np.einsum("hwc,vh->vwc", x, K) + (1 << (PREC - 1))).astype(np.int64)
    return x.astype(np.uint8)


def pil_crop(img, left, up, ow, oh):
    """Image.crop((left, up, left + ow, up + oh)): pixels outside the image are 0."""
    h, w = img.shape[:2]
    out = np.zeros((oh, ow) + img.shape[2:], img.dtype)
    y0, y1 = max(up, 0), min(up + oh, h)
    x0, x1 = max(left, 0), min(left + ow, w)
    if y1 > y0 and x1 > x0:
        out[y0 - up:y1 - up, x0 - left:x1 - left] = img[y0:y1, x0:x1]
    return out


def pil_resize_crop(img, box, oh=224, ow=224, kind=3):
    w, h, left, up = box
    return pil_crop(pil_resize(img, w, h, kind), left, up, ow, oh)


# ----------------------------------------------------------------------------- alignment
def lm3d_5p(lm3d):
    """load_mats.py:110-114."""
    idx = np.array([31, 37, 40, 43, 46, 49, 55]) - 1
    out = np.stack([lm3d[idx[0], :], np.mean(lm3d[idx[[1, 2]], :], 0), np.mean(lm3d[idx[[3, 4]], :], 0),
                    lm3d[idx[5], :], lm3d[idx[6], :]], axis=0)
    return out[[1, 2, 0, 3, 4], :]


extract_5p = lm3d_5p                                 # preprocess.py:173-179 is the same reduction


def pos(xp, x):
    """preprocess.py:18-43."""
    n = xp.shape[1]
    A = np.zeros([2 * n, 8])
    A[0:2 * n - 1:2, 0:3] = x.T
    A[0:2 * n - 1:2, 3] = 1
    A[1:2 * n:2, 4:7] = x.T
    A[1:2 * n:2, 7] = 1
    b = np.reshape(xp.T, [2 * n, 1])
    k = np.linalg.lstsq(A, b, rcond=None)[0]
    s = (np.linalg.norm(k[0:3]) + np.linalg.norm(k[4:7])) / 2
    return np.stack([k[3], k[7]], axis=0), s


def align(w0, h0, lm, lm3d, target=224.0, rescale=102.0):
    """align_img + resize_n_crop_img geometry -> (trans_params [5], (w, h, left, up), lm_new)."""
    lm5 = extract_5p(lm) if lm.shape[0] != 5 else lm
    t, s = pos(lm5.T, lm3d.T)
    s = rescale / s
    w, h = int(np.int32(w0 * s)), int(np.int32(h0 * s))
    left = int(np.float64(w / 2 - target / 2 + float(((t[0] - w0 / 2) * s)[0])).astype(np.int32))
    up = int(np.float64(h / 2 - target / 2 + float(((h0 / 2 - t[1]) * s)[0])).astype(np.int32))
    lm_new = np.stack([lm[:, 0] - t[0] + w0 / 2, lm[:, 1] - t[1] + h0 / 2], axis=1) * s
    lm_new = lm_new - np.array([[w / 2 - target / 2, h / 2 - target / 2]])
    return np.array([w0, h0, s, t[0, 0], t[1, 0]], np.float64), (w, h, left, up), lm_new


# ----------------------------------------------------------------------------- network
def recon_forward(sd, x):
    """x [B,3,H,W] float (RGB / 255) -> [B, 257] (networks.py:98-105, use_last_fc=False)."""
    y = resnet50_body(sd, x, p="backbone.")[-1]
    y = F.adaptive_avg_pool2d(y, (1, 1))
    outs = [F.conv2d(y, sd[f"final_layers.{i}.weight"], sd[f"final_layers.{i}.bias"]) for i in range(7)]
    return torch.flatten(torch.cat(outs, 1), 1)


def face_3dmm_extraction(sd, frames, lms, lm3d):
    """facing.py:108-129 for RGB uint8 frames [N,H,W,3] and landmarks [N,68,2] -> [N, 262] float32."""
    rows = []
    for img, lm in zip(frames, lms):
        H, W = img.shape[:2]
        li = np.array(lm, np.float32).reshape([-1, 2])
        if np.mean(li) == -1:
            li = (lm3d[:, :2] + 1) / 2.
            li = np.concatenate([li[:, :1] * W, li[:, 1:2] * H], 1)
        else:
            li[:, -1] = H - 1 - li[:, -1]
        trans, box, _ = align(W, H, li, lm3d)
        im = pil_resize_crop(img, box)
        x = torch.tensor(np.array(im) / 255., dtype=torch.float32).permute(2, 0, 1)[None]
        with torch.no_grad():
            c = recon_forward(sd, x).numpy()
        rows.append(np.concatenate([c[:, :80], c[:, 80:144], c[:, 144:224], c[:, 224:227], c[:, 227:254], c[:, 254:],
                                    trans.astype(np.float32)[None]], 1))
    return np.concatenate(rows, 0)
