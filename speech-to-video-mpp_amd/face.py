"""Face detection, alignment and GPEN's FaceEnhancement on the device (SURVEY.md §8f(3) and the
§8f(2) composition): drop-ins for

    third_part/GPEN/face_detect/retinaface_detection.py:19-124   RetinaFaceDetection(.detect)
    third_part/GPEN/align_faces.py:103-266                       get_reference_facial_points,
                                                                 warp_and_crop_face
    third_part/GPEN/face_model/face_gan.py:13-59                 FaceGAN(.process)
    third_part/GPEN/face_enhancement.py:49-193                   FaceEnhancement(.process)

    from s2v_amd import face
    enhancer = face.FaceEnhancement(args, base_dir='checkpoints', in_size=2048, model='GPEN-BFR-2048',
                                    use_sr=True, sr_scale=2, sr_model=None)        # inference.py:228-231
    pp, orig_faces, enhanced_faces = enhancer.process(pp, tmp_xf, bbox=c, face_enhance=True,
                                                      possion_blending=True)       # inference.py:319

Images are uint8 HWC BGR (NumPy arrays are copied to the device; ``process_device`` keeps device
tensors end to end).  On the device: the RetinaFace-R50 network and its prior decode + threshold
(s2v_retina_decode), every cv2.warpAffine / resize / GaussianBlur / filter2D, FaceGAN's tensor
conversions, GPEN, RealESRNet, ParseNet, the paste-back composite and the final blends.  On the host,
as in the reference: the NMS over the few thresholded candidates, the 5-point similarity fit
(Umeyama, 5x2 points) and the per-face loop.  There is no CPU path.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

from . import ops, post
from ._lib import check
from .ops import NHWC

CFG_VARIANCE = (0.1, 0.2)
FACE_MM = [0, 255, 255, 255, 255, 255, 255, 255, 0, 0, 255, 255, 255, 0, 0, 0, 0, 0, 0]   # face_enhancement.py:136
SMALL_FACE_KERNEL = ((0.0625, 0.125, 0.0625), (0.125, 0.25, 0.125), (0.0625, 0.125, 0.0625))   # :67-70

WARP_DTYPES = {torch.uint8: 0, torch.float32: 1, torch.float64: 2}


def _ctx(device):
    return post._ctx(device)


def _frame(img, device) -> torch.Tensor:
    t = post.to_device(img, device)
    if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
        raise TypeError(f"expected a uint8 HWC BGR frame, got {tuple(t.shape)} {t.dtype}")
    return t.contiguous()


# ----------------------------------------------------------------------------- alignment (host)
REFERENCE_FACIAL_POINTS = [[30.29459953, 51.69630051], [65.53179932, 51.50139999], [48.02519989, 71.73660278],
                           [33.54930115, 92.3655014], [62.72990036, 92.20410156]]   # align_faces.py:14-20
DEFAULT_CROP_SIZE = (96, 112)


class FaceWarpException(Exception):
    pass


def get_reference_facial_points(output_size=None, inner_padding_factor=0.0, outer_padding=(0, 0),
                                default_square=False):
    """align_faces.py:103-195: the 5 reference points for a crop of ``output_size``."""
    tmp_5pts = np.array(REFERENCE_FACIAL_POINTS)
    tmp_crop_size = np.array(DEFAULT_CROP_SIZE)
    if default_square:
        size_diff = max(tmp_crop_size) - tmp_crop_size
        tmp_5pts += size_diff / 2
        tmp_crop_size += size_diff
    if output_size and output_size[0] == tmp_crop_size[0] and output_size[1] == tmp_crop_size[1]:
        return tmp_5pts
    if inner_padding_factor == 0 and outer_padding == (0, 0):
        if output_size is None:
            return tmp_5pts
        raise FaceWarpException(f"No paddings to do, output_size must be None or {tmp_crop_size}")
    if not (0 <= inner_padding_factor <= 1.0):
        raise FaceWarpException("Not (0 <= inner_padding_factor <= 1.0)")
    if (inner_padding_factor > 0 or outer_padding[0] > 0 or outer_padding[1] > 0) and output_size is None:
        output_size = (tmp_crop_size * (1 + inner_padding_factor * 2)).astype(np.int32)
        output_size += np.array(outer_padding)
    if not (outer_padding[0] < output_size[0] and outer_padding[1] < output_size[1]):
        raise FaceWarpException("Not (outer_padding[0] < output_size[0] and outer_padding[1] < output_size[1])")
    if inner_padding_factor > 0:
        size_diff = tmp_crop_size * inner_padding_factor * 2
        tmp_5pts += size_diff / 2
        tmp_crop_size += np.round(size_diff).astype(np.int32)
    size_bf_outer_pad = np.array(output_size) - np.array(outer_padding) * 2
    if size_bf_outer_pad[0] * tmp_crop_size[1] != size_bf_outer_pad[1] * tmp_crop_size[0]:
        raise FaceWarpException("Must have (output_size - outer_padding) = some_scale * (crop_size * (1.0 + "
                                "inner_padding_factor)")
    scale_factor = size_bf_outer_pad[0].astype(np.float32) / tmp_crop_size[0]
    tmp_5pts = tmp_5pts * scale_factor
    return tmp_5pts + np.array(outer_padding)


def _umeyama(src, dst, estimate_scale=True, scale=1.0):
    """Least-squares similarity (Umeyama 1991) as align_faces.py:34-95 computes it (same dtypes)."""
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
    if rank == dim - 1:
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


def _pts(p, what):
    p = np.float32(p)
    if max(p.shape) < 3 or min(p.shape) != 2:
        raise FaceWarpException(f"{what}.shape must be (K,2) or (2,K) and K>2")
    return p.T if p.shape[0] == 2 else p


def similarity_transforms(facial_pts, reference_pts):
    """warp_and_crop_face's 'smilarity' transforms (align_faces.py:230-258) -> (tfm, tfm_inv)."""
    ref_pts, src_pts = _pts(reference_pts, "reference_pts"), _pts(facial_pts, "facial_pts")
    if src_pts.shape != ref_pts.shape:
        raise FaceWarpException("facial_pts and reference_pts must have the same shape")
    params, scale = _umeyama(src_pts, ref_pts)
    tfm = params[:2, :]
    params, _ = _umeyama(ref_pts, src_pts, False, scale=1.0 / scale)
    return tfm, params[:2, :]


# ----------------------------------------------------------------------------- device image ops
def _mats(ms, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(np.asarray(ms, np.float64).reshape(-1, 6))).to(device)


def warp_affine(src: torch.Tensor, M, dsize, out: torch.Tensor | None = None) -> torch.Tensor:
    """cv2.warpAffine(src, M, dsize, flags=INTER_LINEAR | INTER_AREA, BORDER_CONSTANT 0) on a device
    image [H,W] / [H,W,C] (uint8, float32 or float64) or a batch [N,H,W,C] with N matrices."""
    if src.dtype not in WARP_DTYPES:
        raise TypeError(f"warp_affine: {src.dtype} images are not supported")
    n, h, w, c, xrs, xis = post._hwc(src)
    W, H = dsize
    Ms = np.asarray(M, np.float64).reshape(-1, 2, 3)
    if Ms.shape[0] != n:
        raise ValueError(f"warp_affine: {Ms.shape[0]} matrices for {n} images")
    if out is None:
        shape = {2: (H, W), 3: (H, W, c)}.get(src.dim(), (n, H, W, c))
        out = torch.empty(shape, dtype=src.dtype, device=src.device)
    on, oh, ow, oc, yrs, yis = post._hwc(out)
    if (on, oh, ow, oc) != (n, H, W, c) or out.dtype != src.dtype:
        raise ValueError("warp_affine: output view does not match")
    ctx = _ctx(src.device)
    md = _mats(Ms, src.device)
    check(ctx.lib.s2v_warp_affine(src.data_ptr(), n, h, w, c, xrs, xis, WARP_DTYPES[src.dtype], md.data_ptr(),
                                  out.data_ptr(), H, W, yrs, yis, ctx.stream), "s2v_warp_affine")
    return out


def warp_and_crop_face(src_img, facial_pts, reference_pts=None, crop_size=(96, 112), align_type="smilarity"):
    """align_faces.py:210-266 (the 'smilarity' alignment FaceEnhancement uses) -> (face_img device
    uint8, tfm_inv)."""
    if align_type != "smilarity":
        raise NotImplementedError("warp_and_crop_face: only the 'smilarity' alignment is on the GPEN path")
    if reference_pts is None:
        if tuple(crop_size) == (96, 112):
            reference_pts = REFERENCE_FACIAL_POINTS
        else:
            reference_pts = get_reference_facial_points(crop_size, 0, (0, 0), False)
    src = post.to_device(src_img, "cuda" if not isinstance(src_img, torch.Tensor) else src_img.device)
    tfm, tfm_inv = similarity_transforms(facial_pts, reference_pts)
    return warp_affine(src, tfm, (crop_size[0], crop_size[1])), tfm_inv


_KERNELS = {}


def _gauss_taps(ksize, sigma, dtype, device) -> torch.Tensor:
    """cv::getGaussianKernel (bit-exact form: see oracle/face.py gaussian_kernel) on the device."""
    key = (ksize, float(sigma), dtype, str(device))
    if key not in _KERNELS:
        n = ksize if ksize > 0 else int(np.rint(sigma * 8 + 1)) | 1
        scale2x = -0.125 / (sigma * sigma)
        vals, tot = [], 0.0
        for i in range((n - 1) // 2):
            x = 1 - n + 2 * i
            t = math.exp(float(x * x) * scale2x)
            vals.append(t)
            tot += t
        mul = 1.0 / (tot * 2.0 + 1.0)
        k = [v * mul for v in vals]
        taps = np.array(k + [1.0 * mul] + k[::-1], np.float64).astype(np.float32 if dtype == 1 else np.float64)
        _KERNELS[key] = torch.from_numpy(taps).to(device)
    return _KERNELS[key]


def gaussian_blur(x: torch.Tensor, ksize, sigma, *, out_dtype=None, zero_border=0, u8_scale=False) -> torch.Tensor:
    """cv2.GaussianBlur(x, (ksize, ksize), sigma) on a [H,W] float32 / float64 device image
    (BORDER_REFLECT_101).  ``u8_scale``: x is uint8 and the blurred image is x / 255. (float64);
    ``zero_border``: the input is zeroed outside [zb, H-zb) x [zb, W-zb) first."""
    h, w = x.shape
    dt = 2 if (u8_scale or x.dtype == torch.float64) else 1
    xt = 0 if u8_scale else dt
    if u8_scale and x.dtype != torch.uint8:
        raise TypeError("gaussian_blur: u8_scale takes a uint8 mask")
    out_dtype = out_dtype or (torch.float64 if dt == 2 else torch.float32)
    y = torch.empty((h, w), dtype=out_dtype, device=x.device)
    ctx = _ctx(x.device)
    taps = _gauss_taps(ksize, sigma, dt, x.device)
    need = ctx.lib.s2v_gaussian_blur_ws_bytes(h, w, dt)
    ws, wsb = ctx.ws.get(need)
    check(ctx.lib.s2v_gaussian_blur(x.contiguous().data_ptr(), xt, h, w, zero_border, taps.data_ptr(), taps.numel(),
                                    y.data_ptr(), 2 if out_dtype == torch.float64 else 1, dt, ws, wsb, ctx.stream),
          "s2v_gaussian_blur")
    return y


MASK_BORDER = 26          # FaceEnhancement.mask_postprocess(mask, thres=26) (face_enhancement.py:83)


def mask_postprocess(mask_u8: torch.Tensor, thres=MASK_BORDER) -> torch.Tensor:
    """FaceEnhancement.mask_postprocess (face_enhancement.py:83-88) of mask_sharp = parse / 255.:
    border zeroing + /255 fused into the first blur's row pass, two 101-tap sigma-11 blurs in fp64,
    astype(float32) fused into the second's column pass."""
    t = gaussian_blur(mask_u8, 101, 11, zero_border=thres, u8_scale=True)
    return gaussian_blur(t, 101, 11, out_dtype=torch.float32)


_SMALL_K = {}


def filter2d_smooth(img: torch.Tensor) -> torch.Tensor:
    """cv2.filter2D(ef, -1, self.kernel) on a uint8 HWC face (face_enhancement.py:159-160)."""
    key = str(img.device)
    if key not in _SMALL_K:
        _SMALL_K[key] = torch.tensor(SMALL_FACE_KERNEL, dtype=torch.float32).reshape(-1).to(img.device)
    h, w, c = img.shape
    y = torch.empty_like(img)
    ctx = _ctx(img.device)
    check(ctx.lib.s2v_filter3x3_u8(img.contiguous().data_ptr(), h, w, c, _SMALL_K[key].data_ptr(), y.data_ptr(),
                                   ctx.stream), "s2v_filter3x3_u8")
    return y


# ----------------------------------------------------------------------------- detection
class RetinaFaceDetection:
    """retinaface_detection.py:19-124 on the device.  ``net``: an s2v_amd.models.RetinaFace; without
    it the weights load from base_dir/weights/<network>.pth."""

    def __init__(self, base_dir="./", device="cuda", network="RetinaFace-R50", net=None):
        from . import models
        self.device = torch.device(device)
        self.cfg = dict(models.retinaface_arch.CFG_RE50)
        self.pretrained_path = os.path.join(base_dir, "weights", network + ".pth")
        self.net = net.eval() if net is not None else models.load_retinaface(self.pretrained_path)
        self._cand = None

    def head_maps(self, img: torch.Tensor):
        """Device uint8 (or float32 resized) frame [H,W,3] -> per-level fused head maps."""
        h, w = img.shape[:2]
        x4 = NHWC.empty(1, h, w, 4, self.device)
        ctx = _ctx(self.device)
        check(ctx.lib.s2v_bgr_mean_nhwc4(img.contiguous().data_ptr(), 0 if img.dtype == torch.uint8 else 1, h * w,
                                         x4.ptr, ctx.stream), "s2v_bgr_mean_nhwc4")
        maps, _ = self.net.head_maps(x4)
        return maps

    def candidates(self, maps, im_h, im_w, confidence_threshold):
        """Priors whose score > threshold, as the reference's thresholded arrays in prior order:
        (boxes [K,4], scores [K], landms [K,10]) float32 NumPy (one device -> host copy of K rows)."""
        P = sum(2 * m.h * m.w for m in maps)
        if self._cand is None or self._cand[0].numel() < P * 16:
            self._cand = (torch.empty(P * 16, device=self.device), torch.empty(1, dtype=torch.int32, device=self.device))
        cand, count = self._cand
        ctx = _ctx(self.device)
        heads = (ctypes.c_void_p * 3)(*[m.ptr for m in maps])
        hs = (ctypes.c_int * 3)(*[m.h for m in maps])
        ws = (ctypes.c_int * 3)(*[m.w for m in maps])
        check(ctx.lib.s2v_retina_decode(heads, hs, ws, maps[0].cs, im_h, im_w, float(confidence_threshold),
                                        cand.data_ptr(), count.data_ptr(), cand.numel() // 16, ctx.stream),
              "s2v_retina_decode")
        k = int(count.item())
        rows = cand[: k * 16].view(k, 16).cpu().numpy()
        rows = rows[np.argsort(rows[:, 0].view(np.int32), kind="stable")]
        return rows[:, 1:5].copy(), rows[:, 5].copy(), rows[:, 6:16].copy()

    def detect(self, img_raw, resize=1, confidence_threshold=0.9, nms_threshold=0.4, top_k=5000, keep_top_k=750,
               save_image=False):
        """-> (dets [K,5] float32 x1 y1 x2 y2 score, landms [K,10] x0..x4 y0..y4), as the reference."""
        img = _frame(img_raw, self.device)
        im_height, im_width = img.shape[:2]
        ss = 1.0
        if max(im_height, im_width) > 1500:                         # "tricky" (:66-70)
            ss = 1000.0 / max(im_height, im_width)
            oh, ow = int(np.rint(im_height * ss)), int(np.rint(im_width * ss))
            img = post.resize_linear(img.float(), (ow, oh), fxfy=(ss, ss))
            im_height, im_width = oh, ow
        maps = self.head_maps(img)
        boxes, scores, landms = self.candidates(maps, im_height, im_width, confidence_threshold)
        if resize != 1:
            boxes, landms = boxes / resize, landms / resize
        return nms_postprocess(boxes, scores, landms, nms_threshold, top_k, keep_top_k, ss)


def py_cpu_nms(dets, thresh):
    """Greedy NMS (utils/nms/py_cpu_nms.py:10-37) over the thresholded candidates (host)."""
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
        inter = np.maximum(0.0, xx2 - xx1 + 1) * np.maximum(0.0, yy2 - yy1 + 1)
        ovr = inter / (areas[i] + areas[order[1:]] - inter)
        order = order[np.where(ovr <= thresh)[0] + 1]
    return keep


def nms_postprocess(boxes, scores, landms, nms_threshold=0.4, top_k=5000, keep_top_k=750, ss=1.0):
    """retinaface_detection.py:105-131 on the thresholded candidates (in prior order)."""
    order = scores.argsort()[::-1][:top_k]
    boxes, landms, scores = boxes[order], landms[order], scores[order]
    dets = np.hstack((boxes, scores[:, np.newaxis])).astype(np.float32, copy=False)
    keep = py_cpu_nms(dets, nms_threshold)
    dets, landms = dets[keep, :][:keep_top_k, :], landms[keep][:keep_top_k, :]
    landms = landms.reshape((-1, 5, 2)).transpose((0, 2, 1)).reshape(-1, 10)
    return dets / ss, landms / ss


# ----------------------------------------------------------------------------- GPEN face GAN
class FaceGAN:
    """face_gan.py:13-59 on the device: cv2.resize to in_size, img2tensor, FullGenerator, tensor2img.
    ``net``: an s2v_amd.models.FullGenerator; without it the weights load from base_dir/weights."""

    def __init__(self, base_dir="./", in_size=512, out_size=None, model=None, channel_multiplier=2, narrow=1,
                 key=None, is_norm=True, device="cuda", net=None):
        from . import models
        if not is_norm:
            raise NotImplementedError("FaceGAN: is_norm=False is not on the FaceEnhancement path")
        self.device = torch.device(device)
        self.in_resolution = in_size
        self.out_resolution = in_size if out_size is None else out_size
        if self.out_resolution != self.in_resolution:
            raise NotImplementedError("FaceGAN: FullGenerator_SR (out_size != in_size) is not on the CLI path")
        if net is None:
            net = models.load_gpen(os.path.join(base_dir, "weights", model + ".pth"), in_size, channel_multiplier,
                                   narrow, key)
        self.model = net.eval()

    def process_device(self, faces: torch.Tensor) -> torch.Tensor:
        """[N,S,S,3] (or [S,S,3]) uint8 BGR device faces -> the same shape uint8 (S = in_size)."""
        single = faces.dim() == 3
        if single:
            faces = faces.unsqueeze(0)
        n, h, w, _ = faces.shape
        S = self.in_resolution
        if (h, w) != (S, S):
            faces = post.resize_linear(faces.contiguous(), (S, S))
        ctx = _ctx(self.device)
        x = torch.empty((n, 3, S, S), device=self.device)
        check(ctx.lib.s2v_u8_to_gan(faces.contiguous().data_ptr(), n, S, S, x.data_ptr(), ctx.stream), "s2v_u8_to_gan")
        eng, ectx = self.model._engine(self.device)
        y = torch.empty_like(x)
        eng.forward(ectx, x, y)
        out = torch.empty((n, S, S, 3), dtype=torch.uint8, device=self.device)
        check(ctx.lib.s2v_gan_to_u8(y.data_ptr(), n, S, S, out.data_ptr(), ctx.stream), "s2v_gan_to_u8")
        return out[0] if single else out

    @torch.no_grad()
    def process(self, img):
        return self.process_device(_frame(img, self.device)).cpu().numpy()


# ----------------------------------------------------------------------------- FaceEnhancement
class FaceEnhancement:
    """face_enhancement.py:49-193.  The networks load from base_dir/weights as in the reference, or
    are given (``facedetector`` / ``facegan`` / ``srmodel`` / ``faceparser``: this module's
    RetinaFaceDetection / FaceGAN, s2v_amd.sr.RealESRNet, s2v_amd.post.FaceParse)."""

    def __init__(self, args=None, base_dir="./", in_size=1024, out_size=None, model=None, use_sr=True, device="cuda",
                 sr_scale=4, sr_model="rrdb_realesrnet_psnr", channel_multiplier=2, narrow=1, *, facedetector=None,
                 facegan=None, srmodel=None, faceparser=None):
        from . import sr
        self.device = torch.device(device)
        self.sr_scale = sr_scale
        self.facedetector = facedetector or RetinaFaceDetection(base_dir, device)
        self.facegan = facegan or FaceGAN(base_dir, in_size, out_size, model, channel_multiplier, narrow, None,
                                          device=device)
        self.srmodel = srmodel if srmodel is not None else (
            sr.RealESRNet(base_dir, sr_model, scale=sr_scale, tile_size=0, device=device) if use_sr else None)
        self.faceparser = faceparser or post.FaceParse(base_dir, device=device)
        self.use_sr = use_sr
        self.in_size = in_size
        self.out_size = in_size if out_size is None else out_size
        if self.out_size != self.in_size:
            raise NotImplementedError("FaceEnhancement: out_size != in_size is not on the CLI path")
        self.threshold = 0.9
        self.alpha = 1.0                     # cv2.addWeighted(ef, 1.0, of, 0.0, 0.0) is the identity
        self.reference_5pts = get_reference_facial_points((self.in_size, self.in_size), 0.25, (0, 0), True)

    def _parse(self, ef: torch.Tensor) -> torch.Tensor:
        """FaceParse.process(ef, FACE_MM)[0]: uint8 512x512 mask of the (resized) face."""
        S = self.faceparser.size
        im = ef if ef.shape[0] == S else post.resize_linear(ef, (S, S))
        return self.faceparser.masks_device(im, FACE_MM)[0]

    @torch.no_grad()
    def process_device(self, img, ori_img, face_enhance=True, bbox=None, possion_blending=False, trace=None):
        """FaceEnhancement.process on device frames -> (uint8 [H,W,3] device frame, orig_faces,
        enhanced_faces as device tensors).  ``trace`` (a dict) receives the per-face intermediates
        (detections, parse masks, faces) for the composition tests."""
        dev = self.device
        img, ori = _frame(img, dev), _frame(ori_img, dev)
        orig_faces, enhanced_faces = [], []
        img_sr = None
        if self.use_sr:
            try:
                img_sr = self.srmodel.process_device(img)
            except Exception as e:  # noqa: BLE001 - RealESRNet.process's contract (real_esrnet.py:136-137)
                print("sr failed:", e)
                img_sr = None
            if img_sr is not None:
                img = post.resize_linear(img, (img_sr.shape[1], img_sr.shape[0]))
        facebs, landms = self.facedetector.detect(img)
        height, width = img.shape[:2]
        ctx = _ctx(dev)
        full_mask = torch.zeros((height, width), dtype=torch.float32, device=dev)
        full_img = torch.zeros(ori.shape, dtype=torch.uint8, device=dev)
        if full_img.shape[:2] != (height, width):
            raise ValueError(f"FaceEnhancement: ori_img {tuple(ori.shape)} must match the (super-resolved) frame "
                             f"{(height, width)} (the reference's full_img[mask > 0] = tmp_img[...] needs it)")
        S = self.in_size
        need_sharp = not (self.use_sr and img_sr is not None)        # mask_sharp only feeds the non-SR blends
        mask_sharp = None
        if trace is not None:
            trace.update(dets=facebs, landms=landms, img_sr=img_sr, img=img, masks=[])
        for faceb, facial5points in zip(facebs, landms):
            if faceb[4] < self.threshold:
                continue
            fh, fw = (faceb[3] - faceb[1]), (faceb[2] - faceb[0])
            tfm, tfm_inv = similarity_transforms(np.reshape(facial5points, (2, 5)), self.reference_5pts)
            of = warp_affine(img, tfm, (S, S))
            ef = self.facegan.process_device(of) if face_enhance else of
            orig_faces.append(of)
            enhanced_faces.append(ef)           # before the small-face filter, as the reference appends it
            m8 = self._parse(ef)
            tmp_mask = mask_postprocess(m8)
            if tmp_mask.shape[0] != S:
                tmp_mask = post.resize_linear(tmp_mask, (S, S))
            if need_sharp:
                # mask_sharp = parse / 255. as mask_postprocess left it: the reference zeroes its
                # 26-pixel border IN PLACE (face_enhancement.py:84-85 on the array of :144) before it
                # is resized and warped (:149-150)
                ms = torch.empty(m8.shape, dtype=torch.float64, device=dev)
                check(ctx.lib.s2v_u8_div255_f64_border(m8.data_ptr(), m8.shape[0], m8.shape[1], MASK_BORDER,
                                                       ms.data_ptr(), ctx.stream), "s2v_u8_div255_f64_border")
                if ms.shape[0] != ef.shape[0]:
                    ms = post.resize_linear(ms, (ef.shape[1], ef.shape[0]))
                mask_sharp = warp_affine(ms, tfm_inv, (width, height))
            else:
                mask_sharp = True
            if min(fh, fw) < 100:
                ef = filter2d_smooth(ef)
            y0, x0, wh, ww = paste_window(tfm_inv, S, height, width)
            md = _mats(tfm_inv, dev)
            check(ctx.lib.s2v_face_paste(tmp_mask.data_ptr(), ef.contiguous().data_ptr(), S, md.data_ptr(),
                                         full_mask.data_ptr(), full_img.data_ptr(), height, width, y0, x0, wh, ww,
                                         ctx.stream), "s2v_face_paste")
            if trace is not None:
                trace["masks"].append(m8)
        if mask_sharp is None:
            raise UnboundLocalError("local variable 'mask_sharp' referenced before assignment (no face above the "
                                    "threshold: face_enhancement.py:165 fails the same way)")
        out = torch.empty(ori.shape, dtype=torch.uint8, device=dev)
        if not need_sharp:
            check(ctx.lib.s2v_face_blend(img_sr.data_ptr(), full_mask.data_ptr(), full_img.data_ptr(), None,
                                         out.data_ptr(), height * width, ctx.stream), "s2v_face_blend")
            return out, orig_faces, enhanced_faces
        mask_sharp = gaussian_blur(mask_sharp, 0, 1.0)
        if possion_blending:
            if bbox is not None:
                y1, y2, x1, x2 = bbox
                m = torch.zeros((height, width), dtype=torch.float32, device=dev)
                m[y1:y2 - 5, x1:x2] = mask_sharp[y1:y2 - 5, x1:x2].float()     # np.float32(mask_sharp * mask_bbox)
            else:
                m = full_mask
            A, B = post.resize_linear(full_img, (512, 512)), post.resize_linear(ori, (512, 512))
            M = post.resize_linear(m.contiguous(), (512, 512))
            blended = post.laplacian_pyramid_blending_with_mask(A, B, M, 6, clip=True)
            return post.resize_linear(blended, (width, height), out=out, mode=post.RS_F32_TO_U8), orig_faces, \
                enhanced_faces
        check(ctx.lib.s2v_face_blend(ori.data_ptr(), full_mask.data_ptr(), full_img.data_ptr(), mask_sharp.data_ptr(),
                                     out.data_ptr(), height * width, ctx.stream), "s2v_face_blend")
        return out, orig_faces, enhanced_faces

    def mask_postprocess(self, mask, thres=26):
        """face_enhancement.py:83-88 on a uint8 parse mask (mask_sharp * 255) -> float32 device mask."""
        return mask_postprocess(post.to_device(mask, self.device), thres)

    @torch.no_grad()
    def process(self, img, ori_img, face_enhance=True, bbox=None, possion_blending=False):
        """face_enhancement.py:91-193: NumPy / device uint8 frames -> (img NumPy uint8, orig_faces,
        enhanced_faces as NumPy uint8 lists), as the reference returns them."""
        out, of, ef = self.process_device(img, ori_img, face_enhance, bbox, possion_blending)
        return out.cpu().numpy(), [f.cpu().numpy() for f in of], [f.cpu().numpy() for f in ef]


def paste_window(tfm_inv, S, H, W):
    """Frame window [y0, y0+wh) x [x0, x0+ww) holding every pixel whose warped crop value can be
    non-zero: the image of the crop square (-1, S) x (-1, S) under tfm_inv, padded for the
    fixed-point coordinate rounding.  Outside it the warped mask is exactly 0, which never exceeds
    the running full mask, so the paste writes nothing there (face_enhancement.py:155-157)."""
    M = np.asarray(tfm_inv, np.float64)
    cs = np.array([[-2.0, -2.0], [S + 1.0, -2.0], [-2.0, S + 1.0], [S + 1.0, S + 1.0]])
    p = cs @ M[:, :2].T + M[:, 2]
    pad = 2.0 + 2.0 * max(1.0, float(np.abs(M[:, :2]).sum(1).max()))
    x0, y0 = int(max(0, np.floor(p[:, 0].min() - pad))), int(max(0, np.floor(p[:, 1].min() - pad)))
    x1, y1 = int(min(W, np.ceil(p[:, 0].max() + pad))), int(min(H, np.ceil(p[:, 1].max() + pad)))
    return y0, x0, max(0, y1 - y0), max(0, x1 - x0)
