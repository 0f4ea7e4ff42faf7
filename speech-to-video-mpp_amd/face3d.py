"""3DMM coefficient extraction that feeds DNet: the per-frame loop of
preprocessing/facing.py:100-130 (face_3dmm_extraction) and :136-165 (hack_3dmm_expression from an
image), batched over the whole clip on the device.

Reference chain per frame (facing.py:108-127):
    lm (68 FAN landmarks, or all -1 when none was found) -> y flipped (H - 1 - y)
    align_img (third_part/face3d/util/preprocess.py:186-216): POS least squares of the 5 landmark
      points against the BFM's lm3D -> scale s, translation t -> resize_n_crop_img (:147-167):
      PIL img.resize((w0*s, h0*s), BICUBIC).crop(224 x 224 window)
    np.array(im) / 255. -> ReconNetWrapper(resnet50) -> split_coeff -> [id, exp, tex, angle, gamma,
      trans, trans_params] = one 262-float row of ``semantic_npy``.

Here the 5-point POS fits (a 10 x 8 least-squares problem per frame) stay on the host, like NMS;
the resize + crop of every frame runs in one s2v_pil_resize_crop launch per batch (Pillow's
fixed-point arithmetic, bit-exact) straight into the NHWC input of the ResNet-50 engine.  The FAN
landmark detector (the face_alignment package) is not part of the reference tree and not
installed: landmarks are an input here, as the reference's own cache file ``*_landmarks.txt`` is.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import ops
from ._lib import check
from .ops import NHWC

TARGET = 224
RESCALE = 102.0
PIL_BILINEAR, PIL_BICUBIC = 2, 3
MAX_DOWNSCALE = 11.5        # s2v_pil_resize_crop: at most 48 taps per output coordinate


def load_lm3d(bfm_folder):
    """util/load_mats.py:105-116: the 5 standard 3D landmarks from BFM's similarity_Lm3D_all.mat."""
    from scipy.io import loadmat
    lm3d = loadmat(os.path.join(bfm_folder, "similarity_Lm3D_all.mat"))["lm"]
    return lm3d_from_68(lm3d)


def lm3d_from_68(lm3d):
    idx = np.array([31, 37, 40, 43, 46, 49, 55]) - 1
    out = np.stack([lm3d[idx[0], :], np.mean(lm3d[idx[[1, 2]], :], 0), np.mean(lm3d[idx[[3, 4]], :], 0),
                    lm3d[idx[5], :], lm3d[idx[6], :]], axis=0)
    return out[[1, 2, 0, 3, 4], :]


def extract_5p(lm):
    """preprocess.py:173-179."""
    idx = np.array([31, 37, 40, 43, 46, 49, 55]) - 1
    p = np.stack([lm[idx[0], :], np.mean(lm[idx[[1, 2]], :], 0), np.mean(lm[idx[[3, 4]], :], 0), lm[idx[5], :],
                  lm[idx[6], :]], axis=0)
    return p[[1, 2, 0, 3, 4], :]


def POS(xp, x):
    """preprocess.py:18-43: least-squares scale + translation of the 3D points x onto xp."""
    npts = xp.shape[1]
    A = np.zeros([2 * npts, 8])
    A[0:2 * npts - 1:2, 0:3] = x.transpose()
    A[0:2 * npts - 1:2, 3] = 1
    A[1:2 * npts:2, 4:7] = x.transpose()
    A[1:2 * npts:2, 7] = 1
    b = np.reshape(xp.transpose(), [2 * npts, 1])
    k, _, _, _ = np.linalg.lstsq(A, b, rcond=None)
    R1, R2 = k[0:3], k[4:7]
    s = (np.linalg.norm(R1) + np.linalg.norm(R2)) / 2
    return np.stack([k[3], k[7]], axis=0), s


def align_params(w0, h0, lm, lm3D, target_size=float(TARGET), rescale_factor=RESCALE):
    """align_img (preprocess.py:186-216) without the pixels: -> (trans_params [w0, h0, s, tx, ty]
    float64, (w, h, left, up) of resize_n_crop_img (:147-158), lm_new)."""
    lm5p = extract_5p(lm) if lm.shape[0] != 5 else lm
    t, s = POS(lm5p.transpose(), lm3D.transpose())
    s = rescale_factor / s
    # resize_n_crop_img: (x).astype(np.int32) truncates toward zero, as int() does
    w = int(w0 * s)
    h = int(h0 * s)
    left = int(w / 2 - target_size / 2 + float(((t[0] - w0 / 2) * s).item()))
    up = int(h / 2 - target_size / 2 + float(((h0 / 2 - t[1]) * s).item()))
    lm_new = np.stack([lm[:, 0] - t[0] + w0 / 2, lm[:, 1] - t[1] + h0 / 2], axis=1) * s
    lm_new = lm_new - np.reshape(np.array([(w / 2 - target_size / 2), (h / 2 - target_size / 2)]), [1, 2])
    trans = np.array([w0, h0, float(s), float(t[0].item()), float(t[1].item())], dtype=np.float64)
    return trans, (w, h, left, up), lm_new


def split_coeff(coeffs):
    """futils/inference_utils.py:158-181."""
    return {"id": coeffs[:, :80], "exp": coeffs[:, 80:144], "tex": coeffs[:, 144:224], "angle": coeffs[:, 224:227],
            "gamma": coeffs[:, 227:254], "trans": coeffs[:, 254:]}


def frame_landmarks(lm, W, H, lm3d_std):
    """facing.py:110-116: the per-frame landmark fix-up before align_img."""
    lm_idx = np.array(lm, dtype=np.float32).reshape([-1, 2])
    if np.mean(lm_idx) == -1:
        lm_idx = (lm3d_std[:, :2] + 1) / 2.
        return np.concatenate([lm_idx[:, :1] * W, lm_idx[:, 1:2] * H], 1)
    lm_idx[:, -1] = H - 1 - lm_idx[:, -1]
    return lm_idx


def _check_scale(w0, h0, w, h):
    if w <= 0 or h <= 0:
        raise ValueError(f"align_img: resized frame {w}x{h} is empty (landmarks too spread for a {w0}x{h0} frame)")
    if w0 / w > MAX_DOWNSCALE or h0 / h > MAX_DOWNSCALE:
        raise ValueError(f"align_img: a {w0}x{h0} -> {w}x{h} bicubic downscale exceeds {MAX_DOWNSCALE}x "
                         "(s2v_pil_resize_crop's 48-tap limit)")


def resize_crop(ctx, frames: torch.Tensor, boxes, out: NHWC, filter=PIL_BICUBIC):
    """PIL resize((w, h)) + crop((left, up, left + ow, up + oh)) of n uint8 RGB frames [n, H, W, 3]
    (device, contiguous) into ``out`` (NHWC fp32, pixel / 255.)."""
    n, H, W, c = frames.shape
    if not (frames.is_cuda and frames.dtype == torch.uint8 and frames.is_contiguous() and c == 3):
        raise ops._lib.S2VError("resize_crop: frames must be a contiguous uint8 [n, H, W, 3] HIP tensor")
    if len(boxes) != n or out.n != n or out.coff != 0:
        raise ValueError("resize_crop: one (w, h, left, up) box and one output image per frame")
    params = box_params(boxes, W, H, frames.device)
    resize_crop_params(ctx, frames, params, out, filter)
    return params


def box_params(boxes, W, H, device):
    """Validated (w, h, left, up) boxes of W x H frames -> the device int32 [n, 4] parameter block."""
    for (w, h, _, _) in boxes:
        _check_scale(W, H, w, h)
    return torch.tensor(np.asarray(boxes, np.int32).reshape(len(boxes), 4), device=device)


def resize_crop_params(ctx, frames: torch.Tensor, params: torch.Tensor, out: NHWC, filter=PIL_BICUBIC):
    """resize_crop with the boxes already on the device (box_params): no host work, graph-capturable."""
    n, H, W, _ = frames.shape
    check(ctx.lib.s2v_pil_resize_crop(frames.data_ptr(), n, H, W, H * W * 3, params.data_ptr(), filter, out.ptr,
                                      out.h, out.w, out.cs, ctx.stream), "s2v_pil_resize_crop")


def align_img(img, lm, lm3D, mask=None, target_size=float(TARGET), rescale_factor=RESCALE):
    """preprocess.py:186-216 on the device: img uint8 HWC RGB tensor -> (trans_params, im_new fp32
    [224, 224, 3] = np.array(img_new) / 255. as facing.py:120 uses it, lm_new, None)."""
    if mask is not None:
        raise NotImplementedError("align_img: the mask branch is training-only (facing.py never passes one)")
    if not isinstance(img, torch.Tensor) or not img.is_cuda:
        raise ops._lib.S2VError("align_img: img must be a uint8 [H, W, 3] HIP tensor (no CPU path)")
    h0, w0 = img.shape[:2]
    trans, box, lm_new = align_params(w0, h0, lm, lm3D, target_size, rescale_factor)
    ctx = ops.Ctx(img.device)
    size = int(target_size)
    out = NHWC.empty(1, size, size, 4, img.device)
    resize_crop(ctx, img.contiguous()[None], [box], out)
    return trans, out.t[0, :, :, :3], lm_new, None


class Face3DExtractor:
    """facing.py:100-130 face_3dmm_extraction (+ :136-165 hack_3dmm_expression's image branch) on a
    ReconNetWrapper: frames in batches of ``batch`` through one resize-crop launch and one ResNet-50
    forward each."""

    def __init__(self, net_recon, lm3d_std, device="cuda", batch=32):
        self.net = net_recon
        self.lm3d = np.asarray(lm3d_std)
        self.device = torch.device(device)
        self.batch = batch
        self.ctx = ops.Ctx(self.device)

    def coeffs(self, frames: torch.Tensor, lms) -> tuple[np.ndarray, np.ndarray]:
        """frames uint8 [N, H, W, 3] RGB on the device, lms [N, 68, 2] (x, y image coordinates, or
        all -1) -> (net_recon coefficients [N, 257] float32, trans_params [N, 5] float32)."""
        N, H, W, _ = frames.shape
        frames = frames.contiguous()
        trans, boxes = [], []
        for i in range(N):
            lm = frame_landmarks(lms[i], W, H, self.lm3d)
            t, box, _ = align_params(W, H, lm, self.lm3d)
            trans.append(np.array([float(v) for v in t], dtype=np.float32))
            boxes.append(box)
        out = torch.empty((N, 257), dtype=torch.float32, device=self.device)
        x4 = NHWC.empty(min(self.batch, N), TARGET, TARGET, 4, self.device)
        for s in range(0, N, self.batch):
            e = min(N, s + self.batch)
            xv = x4 if e - s == x4.n else NHWC(x4.t[: e - s])
            resize_crop(self.ctx, frames[s:e], boxes[s:e], xv)
            out[s:e] = self.net.forward_nhwc(xv)
        torch.cuda.current_stream(self.device).synchronize()
        return out.cpu().numpy(), np.stack(trans)

    def face_3dmm_extraction(self, frames: torch.Tensor, lms) -> np.ndarray:
        """-> semantic_npy [N, 262] float32: [id, exp, tex, angle, gamma, trans, trans_params]
        (facing.py:125-129)."""
        co, trans = self.coeffs(frames, lms)
        c = split_coeff(co)
        return np.concatenate([c["id"], c["exp"], c["tex"], c["angle"], c["gamma"], c["trans"], trans], 1)

    def expression(self, img: torch.Tensor, lm) -> torch.Tensor:
        """hack_3dmm_expression's exp_img branch (facing.py:140-159): the 64 expression coefficients
        of one uint8 RGB image [H, W, 3]."""
        co, _ = self.coeffs(img[None], np.asarray(lm)[None])
        return torch.from_numpy(split_coeff(co)["exp"][0].copy())
