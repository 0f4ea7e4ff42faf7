"""GFPGANer's restore composition on the device: drop-in for

    third_part/GFPGAN/gfpgan/utils.py:19-143   GFPGANer(model_path, upscale, arch='clean', channel_multiplier,
                                               bg_upsampler=None).enhance(img, has_aligned, only_center_face,
                                                                           paste_back)
    facexlib 0.2.5 (requirements.txt:5; not vendored in the reference) utils/face_restoration_helper.py
        FaceRestoreHelper (read_image, get_face_landmarks_5, align_warp_face, get_inverse_affine,
        add_restored_face, paste_faces_to_input_image) and detection/retinaface.py detect_faces

    from s2v_amd.restore import GFPGANer
    restorer = GFPGANer(model_path='checkpoints/GFPGANv1.4.pth', upscale=1, arch='clean',
                        channel_multiplier=2, bg_upsampler=None)                 # inference.py:255-256
    cropped_faces, restored_faces, restored_img = restorer.enhance(
        ff, has_aligned=False, only_center_face=True, paste_back=True)           # inference.py:300-301

Frames are uint8 HWC BGR (NumPy arrays are copied to the device; device tensors stay there).  On the
device: RetinaFace-R50 and its decode + 0.97 threshold (face.RetinaFaceDetection), the 512 x 512
alignment warp with the gray border (s2v_warp_affine_border), img2tensor + normalize (s2v_u8_to_gan),
GFPGANv1Clean for all faces in one batch, tensor2img (s2v_tensor2img_u8), and the paste-back: the
warped square mask with its 2 x 2 erosion and area (s2v_restore_mask), the (2 w_edge)^2 erosion
(s2v_erode_rect_f32), the soft-mask Gaussian blur (s2v_gaussian_blur) and the blend fused with the
face's inverse warp (s2v_restore_paste).  On the host, as in facexlib: the NMS over the thresholded
candidates, the centre-face choice, the 5-point LMEDS similarity fit and the area -> edge width
arithmetic (one 8-byte read-back per face).  There is no CPU path.

Supported as the lip-sync CLI uses it: upscale 1 (the reference's cv2.resize of the background to the
same size is a copy), bg_upsampler None, arch 'clean', FaceRestoreHelper's defaults (5-point template,
no pad_blur, square paste mask: use_parse=False).  oracle/restore.py restates facexlib / OpenCV for
the tests (parity unpinned: neither is importable here).
"""
from __future__ import annotations

import ctypes
import itertools
import math
from fractions import Fraction

import numpy as np
import torch

from . import face as faces
from . import post
from ._lib import check

FFHQ_TEMPLATE_512 = np.array([[192.98138, 239.94708], [318.90277, 240.1936], [256.63416, 314.01935],
                              [201.26117, 371.41043], [313.08905, 371.15118]])   # FaceRestoreHelper.__init__
BORDER_GRAY = (135.0, 133.0, 132.0)        # align_warp_face's borderValue
CONF_THRESHOLD = 0.97                      # get_face_landmarks_5: detect_faces(input_img, 0.97)


# ----------------------------------------------------------------------------- detection
class RetinaFaceDetector:
    """facexlib detection/retinaface.py RetinaFace.detect_faces (use_origin_size=True: no resize) on
    the device network of face.RetinaFaceDetection (same R50 architecture, BGR means 104/117/123)."""

    def __init__(self, base_dir="./", device="cuda", network="RetinaFace-R50", net=None):
        self.det = faces.RetinaFaceDetection(base_dir, device, network, net)
        self.device = self.det.device

    def detect_faces(self, image, conf_threshold=0.8, nms_threshold=0.4, use_origin_size=True):
        """-> [K, 15] float32: x1, y1, x2, y2, score, then the 5 landmarks as interleaved x, y."""
        if not use_origin_size:
            raise NotImplementedError("detect_faces: use_origin_size=False is not on the GFPGANer path")
        img = faces._frame(image, self.device)
        h, w = img.shape[:2]
        maps = self.det.head_maps(img)
        boxes, scores, landms = self.det.candidates(maps, h, w, conf_threshold)
        order = scores.argsort()[::-1]
        boxes, landms, scores = boxes[order], landms[order], scores[order]
        bounding_boxes = np.hstack((boxes, scores[:, np.newaxis])).astype(np.float32, copy=False)
        keep = faces.py_cpu_nms(bounding_boxes, nms_threshold)
        return np.concatenate((bounding_boxes[keep, :], landms[keep]), axis=1)


def edge_boundary(area) -> bool:
    """True when int(sqrt(area)) // 20 (facexlib's w_edge) could change with the last bits of an fp32
    area: sqrt(area) within 1e-4 (relative) of a multiple of 20, where a device sum in another order than
    numpy's pairwise np.sum may land on the other side."""
    r = float(area) ** 0.5
    return r >= 20.0 and abs(r - 20.0 * round(r / 20.0)) <= 1e-4 * r


def get_largest_face(det_faces, h, w):
    """facexlib get_largest_face: the face with the largest box area after clipping the box to the image."""
    def clip(v, n):
        return 0 if v < 0 else (n if v > n else v)
    areas = [(clip(f[2], w) - clip(f[0], w)) * (clip(f[3], h) - clip(f[1], h)) for f in det_faces]
    idx = areas.index(max(areas))
    return det_faces[idx], idx


def get_center_face(det_faces, h=0, w=0, center=None):
    """facexlib get_center_face: the face whose box centre is nearest the image centre."""
    center = np.array(center) if center is not None else np.array([w / 2, h / 2])
    dist = [np.linalg.norm(np.array([(f[0] + f[2]) / 2, (f[1] + f[3]) / 2]) - center) for f in det_faces]
    idx = dist.index(min(dist))
    return det_faces[idx], idx


# ----------------------------------------------------------------------------- similarity fit (host)
def _partial_from_pair(f, t):
    x1, y1, x2, y2 = (float(v) for v in (f[0, 0], f[0, 1], f[1, 0], f[1, 1]))
    X1, Y1, X2, Y2 = (float(v) for v in (t[0, 0], t[0, 1], t[1, 0], t[1, 1]))
    d = 1.0 / ((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2))
    a = d * ((X1 - X2) * (x1 - x2) + (Y1 - Y2) * (y1 - y2))
    b = d * ((Y1 - Y2) * (x1 - x2) - (X1 - X2) * (y1 - y2))
    tx = d * ((Y1 - Y2) * (x1 * y2 - x2 * y1) - (X1 * y2 - X2 * y1) * (y1 - y2) - (X1 * x2 - X2 * x1) * (x1 - x2))
    ty = d * (-(X1 - X2) * (x1 * y2 - x2 * y1) - (Y1 * x2 - Y2 * x1) * (x1 - x2) - (Y1 * y2 - Y2 * y1) * (y1 - y2))
    return np.array([[a, -b, tx], [b, a, ty]])


def _sq_errors(M, f, t):
    ff, tt = f.astype(np.float64), t.astype(np.float64)
    ex = M[0, 0] * ff[:, 0] + M[0, 1] * ff[:, 1] + M[0, 2] - tt[:, 0]
    ey = M[1, 0] * ff[:, 0] + M[1, 1] * ff[:, 1] + M[1, 2] - tt[:, 1]
    return (ex * ex + ey * ey).astype(np.float32)


def estimate_affine_partial_2d(src, dst):
    """cv2.estimateAffinePartial2D(src, dst, method=cv2.LMEDS)[0] for the handful of landmark pairs
    align_warp_face fits: float32 points, 2-point similarity models over every pair (LMeDS keeps the
    lowest median squared error), inliers within OpenCV's LMeDS sigma, then the least-squares 4-DOF
    similarity over the inliers (the optimum of the Levenberg-Marquardt refinement).  None when no
    model exists."""
    f, t = np.float32(src).reshape(-1, 2), np.float32(dst).reshape(-1, 2)
    n = len(f)
    if n < 2:
        return None
    best, best_med = None, math.inf
    for i, j in itertools.combinations(range(n), 2):
        if f[i, 0] == f[j, 0] and f[i, 1] == f[j, 1]:
            continue
        M = _partial_from_pair(f[[i, j]], t[[i, j]])
        if n == 2:
            return M
        med = float(np.sort(_sq_errors(M, f, t))[n // 2])
        if med < best_med:
            best, best_med = M, med
    if best is None:
        return None
    sigma = max(2.5 * 1.4826 * (1 + 5.0 / (n - 2)) * math.sqrt(best_med), 0.001)
    inl = _sq_errors(best, f, t) <= np.float32(sigma * sigma)
    if inl.sum() < 2:
        return None
    fi, ti = f[inl].astype(np.float64), t[inl].astype(np.float64)
    fm, tm = fi.mean(0), ti.mean(0)
    fd, td = fi - fm, ti - tm
    den = (fd * fd).sum()
    a = (fd[:, 0] * td[:, 0] + fd[:, 1] * td[:, 1]).sum() / den
    b = (fd[:, 0] * td[:, 1] - fd[:, 1] * td[:, 0]).sum() / den
    return np.array([[a, -b, tm[0] - (a * fm[0] - b * fm[1])], [b, a, tm[1] - (b * fm[0] + a * fm[1])]])


def invert_affine_transform(M):
    """cv2.invertAffineTransform in double."""
    M = np.asarray(M, np.float64).reshape(2, 3)
    D = M[0, 0] * M[1, 1] - M[0, 1] * M[1, 0]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22, A12, A21 = M[1, 1] * D, M[0, 0] * D, -M[0, 1] * D, -M[1, 0] * D
    return np.array([[A11, A12, -A11 * M[0, 2] - A12 * M[1, 2]], [A21, A22, -A21 * M[0, 2] - A22 * M[1, 2]]])


_TAPS = {}


def gaussian_taps_auto(k, device):
    """getGaussianKernel(k, 0, CV_32F) as GaussianBlur(x, (k, k), 0) builds it (OpenCV 4.x bit-exact
    form): fixed kernels for k = 3, 5, 7; else sigma = k * 0.15 + 0.35 (one rounding), taps as
    face._gauss_taps."""
    key = (k, str(device))
    if key not in _TAPS:
        fixed = {3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
                 7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}
        if k in fixed:
            _TAPS[key] = torch.tensor(fixed[k], dtype=torch.float32, device=device)
        else:
            _TAPS[key] = faces._gauss_taps(k, float(Fraction(k) * Fraction(0.15) + Fraction(0.35)), 1, device)
    return _TAPS[key]


# ----------------------------------------------------------------------------- FaceRestoreHelper
class FaceRestoreHelper:
    """facexlib 0.2.5 FaceRestoreHelper with GFPGANer's arguments (face_size 512, crop_ratio (1, 1),
    det_model 'retinaface_resnet50') on device frames.  ``face_det``: any object with facexlib's
    detect_faces(img, conf_threshold) (RetinaFaceDetector by default)."""

    def __init__(self, upscale_factor, face_size=512, crop_ratio=(1, 1), det_model="retinaface_resnet50",
                 save_ext="png", template_3points=False, pad_blur=False, use_parse=False, device="cuda",
                 face_det=None, base_dir="./"):
        if upscale_factor != 1:
            raise NotImplementedError("FaceRestoreHelper: upscale_factor != 1 (INTER_LANCZOS4 background) is not "
                                      "on the lip-sync path (inference.py:255 uses upscale=1)")
        if template_3points or pad_blur or use_parse or tuple(crop_ratio) != (1, 1):
            raise NotImplementedError("FaceRestoreHelper: only GFPGANer's defaults (5-point template, no pad_blur, "
                                      "square paste mask, crop_ratio (1, 1)) are on the lip-sync path")
        if det_model != "retinaface_resnet50":
            raise NotImplementedError(f"FaceRestoreHelper: detector {det_model!r}")
        self.upscale_factor = upscale_factor
        self.crop_ratio = crop_ratio
        self.face_size = (int(face_size * crop_ratio[1]), face_size)
        self.face_template = FFHQ_TEMPLATE_512 * (face_size / 512.0)
        self.save_ext = save_ext
        self.device = torch.device(device)
        self.face_det = face_det if face_det is not None else RetinaFaceDetector(base_dir, device)
        self.clean_all()

    def clean_all(self):
        self.all_landmarks_5 = []
        self.restored_faces = []
        self.affine_matrices = []
        self.cropped_faces = []
        self.inverse_affine_matrices = []
        self.det_faces = []
        self.input_img = None

    def read_image(self, img):
        """uint8 BGR (HWC, gray HW or BGRA) -> the device input image (HWC BGR)."""
        t = post.to_device(img, self.device)
        if t.dtype != torch.uint8:
            raise TypeError("read_image: 16-bit / float images are not on the lip-sync path")
        if t.dim() == 2:
            t = t.unsqueeze(-1).expand(-1, -1, 3)              # cv2.COLOR_GRAY2BGR
        elif t.shape[2] == 4:
            t = t[:, :, 0:3]
        self.input_img = t.contiguous()

    def get_face_landmarks_5(self, only_keep_largest=False, only_center_face=False, resize=None, blur_ratio=0.01,
                             eye_dist_threshold=None):
        if resize is not None:
            raise NotImplementedError("get_face_landmarks_5: resize is not on the GFPGANer path")
        bboxes = self.face_det.detect_faces(self.input_img, CONF_THRESHOLD)
        for bbox in bboxes:
            # facexlib 0.2.5's expression as published, index quirk included (bbox[5:7] / [7:9] are the eyes;
            # it differences [6]-[8] and [7]-[9]); facexlib is not vendored, so this is restated, parity unpinned
            eye_dist = np.linalg.norm([bbox[6] - bbox[8], bbox[7] - bbox[9]])
            if eye_dist_threshold is not None and eye_dist < eye_dist_threshold:
                continue
            self.all_landmarks_5.append(np.array([[bbox[i], bbox[i + 1]] for i in range(5, 15, 2)]))
            self.det_faces.append(bbox[0:5])
        if len(self.det_faces) == 0:
            return 0
        if only_keep_largest:
            h, w = self.input_img.shape[:2]
            det, idx = get_largest_face(self.det_faces, h, w)
            self.det_faces, self.all_landmarks_5 = [det], [self.all_landmarks_5[idx]]
        elif only_center_face:
            h, w = self.input_img.shape[:2]
            det, idx = get_center_face(self.det_faces, h, w)
            self.det_faces, self.all_landmarks_5 = [det], [self.all_landmarks_5[idx]]
        return len(self.all_landmarks_5)

    def align_warp_face(self, save_cropped_path=None, border_mode="constant"):
        if border_mode != "constant":
            raise NotImplementedError("align_warp_face: only the constant (gray) border is on the GFPGANer path")
        if not self.all_landmarks_5:
            return
        Ms = []
        for lm in self.all_landmarks_5:
            M = estimate_affine_partial_2d(lm, self.face_template)
            if M is None:
                raise RuntimeError("estimateAffinePartial2D found no model (cv2.warpAffine would fail on None)")
            self.affine_matrices.append(M)
            Ms.append(M)
        n, (fw, fh) = len(Ms), self.face_size
        img = self.input_img
        h, w = img.shape[:2]
        out = torch.empty((n, fh, fw, 3), dtype=torch.uint8, device=self.device)
        md = faces._mats(Ms, self.device)
        ctx = faces._ctx(self.device)
        border = (ctypes.c_double * 3)(*BORDER_GRAY)
        check(ctx.lib.s2v_warp_affine_border(img.data_ptr(), n, h, w, 3, w * 3, 0, 0, md.data_ptr(), out.data_ptr(),
                                             fh, fw, fw * 3, fh * fw * 3, border, ctx.stream), "s2v_warp_affine_border")
        self.cropped_faces = list(out.unbind(0))

    def get_inverse_affine(self, save_inverse_affine_path=None):
        for M in self.affine_matrices:
            self.inverse_affine_matrices.append(invert_affine_transform(M) * self.upscale_factor)

    def add_restored_face(self, face):
        self.restored_faces.append(face)

    def paste_faces_to_input_image(self, save_path=None, upsample_img=None, trace=None):
        """-> uint8 [h, w, 3] device frame (``trace``: a list receiving per-face erosion / area /
        w_edge / soft mask for the tests)."""
        if upsample_img is not None:
            raise NotImplementedError("paste_faces_to_input_image: a background upsampler is not on the "
                                      "lip-sync path (bg_upsampler=None)")
        img = self.input_img
        h, w = img.shape[:2]
        assert len(self.restored_faces) == len(self.inverse_affine_matrices), (
            "length of restored_faces and affine_matrices are different.")
        if not self.restored_faces:
            return img.clone()                      # cv2.resize to the same size copies; astype(uint8)
        dev = self.device
        ctx = faces._ctx(dev)
        area = torch.empty(1 + ctx.lib.s2v_restore_parts(), dtype=torch.float64, device=dev)   # result + partials
        acc = None
        out = torch.empty((h, w, 3), dtype=torch.uint8, device=dev)
        S = self.face_size[0]
        last = len(self.restored_faces) - 1
        for i, (face, inv) in enumerate(zip(self.restored_faces, self.inverse_affine_matrices)):
            face = post.to_device(face, dev).contiguous()
            md = faces._mats(inv, dev)
            # the masks are computed on a window: the warped crop's footprint (where inv_mask can be
            # non-zero) padded by the largest erosion + blur reach its area allows (k = 2 w_edge <=
            # sqrt(area) / 10 <= sqrt(footprint) / 10).  Outside it every mask is 0 and the blend is the
            # base itself, and the window's own borders see only zeros, so the result equals the
            # full-frame computation bit for bit.
            fy, fx, fh, fw = faces.paste_window(inv, S, h, w)
            y0 = x0 = wh = ww = 0
            total_face_area, w_edge = np.float32(0.0), 0
            soft = E = None
            if fh > 0 and fw > 0:
                pad = int(math.ceil(math.sqrt(fh * fw) / 10.0)) + 2
                y0, x0 = max(0, fy - pad), max(0, fx - pad)
                wh, ww = min(h, fy + fh + pad) - y0, min(w, fx + fw + pad) - x0
                E = torch.empty((wh, ww), dtype=torch.float32, device=dev)
                C, soft, tmp = torch.empty_like(E), torch.empty_like(E), torch.empty_like(E)
                check(ctx.lib.s2v_restore_mask(md.data_ptr(), S, h, w, y0, x0, wh, ww, E.data_ptr(), area.data_ptr(),
                                               ctx.stream), "s2v_restore_mask")
                total_face_area = np.float32(area[0].item())   # np.sum(inv_mask_erosion) (fp32)
                if edge_boundary(total_face_area):
                    # sqrt(area) within rounding of a multiple of 20: w_edge hangs on the last bits of the
                    # sum, so take it as facexlib does, numpy's pairwise fp32 np.sum over the whole frame
                    full = np.zeros((h, w), dtype=np.float32)
                    full[y0: y0 + wh, x0: x0 + ww] = E.cpu().numpy()
                    total_face_area = np.sum(full)
                w_edge = int(total_face_area ** 0.5) // 20
                k = w_edge * 2
                assert k <= pad, (k, pad)
                check(ctx.lib.s2v_erode_rect_f32(E.data_ptr(), wh, ww, k if k > 0 else 3, C.data_ptr(),
                                                 tmp.data_ptr(), ctx.stream), "s2v_erode_rect_f32")
                if k + 1 == 1:
                    soft.copy_(C)
                else:
                    taps = gaussian_taps_auto(k + 1, dev)
                    need = ctx.lib.s2v_gaussian_blur_ws_bytes(wh, ww, 1)
                    ws, wsb = ctx.ws.get(need)
                    check(ctx.lib.s2v_gaussian_blur(C.data_ptr(), 1, wh, ww, 0, taps.data_ptr(), k + 1,
                                                    soft.data_ptr(), 1, 1, ws, wsb, ctx.stream), "s2v_gaussian_blur")
            if trace is not None:
                trace.append(dict(window=(y0, x0, wh, ww), erosion=None if E is None else E.clone(),
                                  area=total_face_area, w_edge=w_edge, soft=None if soft is None else soft.clone()))
            base, base_f32 = (img, 0) if acc is None else (acc, 1)
            if i == last:
                dst, dst_f32 = out, 0
            else:
                if acc is None:
                    acc = torch.empty((h, w, 3), dtype=torch.float32, device=dev)
                dst, dst_f32 = acc, 1
            sp = soft.data_ptr() if soft is not None else area.data_ptr()      # unread with an empty window
            ep = E.data_ptr() if E is not None else area.data_ptr()
            check(ctx.lib.s2v_restore_paste(face.data_ptr(), S, md.data_ptr(), sp, ep, y0, x0, wh, ww,
                                            base.data_ptr(), base_f32, dst.data_ptr(), dst_f32, h, w, ctx.stream),
                  "s2v_restore_paste")
        return out


# ----------------------------------------------------------------------------- GFPGANer
class GFPGANer:
    """gfpgan/utils.py:19-143 on the device.  ``net``: an s2v_amd.models.GFPGANv1Clean (else the
    weights load from model_path as GFPGANer does); ``face_det``: the detector (see FaceRestoreHelper);
    ``randomize_noise``: the StyleGAN noise of the forward (the reference's default True draws fresh
    noise per call; False uses the stored noise buffers, for deterministic comparisons)."""

    def __init__(self, model_path=None, upscale=2, arch="clean", channel_multiplier=2, bg_upsampler=None,
                 device="cuda", net=None, face_det=None, base_dir="./", randomize_noise=True):
        from . import models
        if arch != "clean":
            raise NotImplementedError(f"GFPGANer: arch {arch!r} (the lip-sync CLI builds arch='clean')")
        if bg_upsampler is not None:
            raise NotImplementedError("GFPGANer: bg_upsampler (inference.py:255 passes None)")
        self.upscale = upscale
        self.bg_upsampler = None
        self.device = torch.device(device)
        self.gfpgan = net.eval() if net is not None else models.load_gfpgan(model_path,
                                                                             channel_multiplier=channel_multiplier)
        self.face_helper = FaceRestoreHelper(upscale, face_size=512, crop_ratio=(1, 1), det_model="retinaface_resnet50",
                                             save_ext="png", device=device, face_det=face_det, base_dir=base_dir)
        self.randomize_noise = randomize_noise

    def _restore(self, cropped):
        """img2tensor + normalize, GFPGANv1Clean(return_rgb=False) over every face at once, tensor2img."""
        x_u8 = torch.stack([post.to_device(f, self.device) for f in cropped]).contiguous()
        n, S = x_u8.shape[0], x_u8.shape[1]
        ctx = faces._ctx(self.device)
        x = torch.empty((n, 3, S, S), device=self.device)
        check(ctx.lib.s2v_u8_to_gan(x_u8.data_ptr(), n, S, S, x.data_ptr(), ctx.stream), "s2v_u8_to_gan")
        try:
            y = self.gfpgan(x, return_rgb=False, randomize_noise=self.randomize_noise)[0]
        except RuntimeError as error:                              # gfpgan/utils.py:122-124
            print(f"\tFailed inference for GFPGAN: {error}.")
            return [f for f in x_u8.unbind(0)]
        out = torch.empty((n, S, S, 3), dtype=torch.uint8, device=self.device)
        check(ctx.lib.s2v_tensor2img_u8(y.contiguous().data_ptr(), n, S, S, out.data_ptr(), ctx.stream),
              "s2v_tensor2img_u8")
        return list(out.unbind(0))

    @torch.no_grad()
    def enhance(self, img, has_aligned=False, only_center_face=False, paste_back=True, trace=None):
        """-> (cropped_faces, restored_faces, restored_img or None), device uint8 tensors."""
        fh = self.face_helper
        fh.clean_all()
        if has_aligned:
            fh.cropped_faces = [post.resize_linear(faces._frame(img, self.device), (512, 512))]
        else:
            fh.read_image(img)
            fh.get_face_landmarks_5(only_center_face=only_center_face, eye_dist_threshold=5)
            fh.align_warp_face()
        if fh.cropped_faces:
            for face in self._restore(fh.cropped_faces):
                fh.add_restored_face(face)
        if not has_aligned and paste_back:
            fh.get_inverse_affine(None)
            restored_img = fh.paste_faces_to_input_image(upsample_img=None, trace=trace)
            return fh.cropped_faces, fh.restored_faces, restored_img
        return fh.cropped_faces, fh.restored_faces, None
