"""Mouth-region post-process on the device: the FaceParse mouth mask and the
Laplacian-pyramid blend that follow ENet + GFPGAN at inference.py:302-313.

    from s2v_amd import models, post
    net = models.load_parsenet("weights/ParseNet-latest.pth")
    parser = post.FaceParse(net=net)
    masks = parser.process(img_u8_bgr, mm)                                  # face_parsing.py:39-45
    img = post.laplacian_pyramid_blending_with_mask(A, B, m, 10)           # inference_utils.py:181-222
    frame = post.MouthBlend(parser).run(restored_img, ff, (y1, y2, x1, x2))  # inference.py:302-313

Images are uint8 HWC (BGR, as cv2 hands them over) device tensors; NumPy arrays are copied to the
device first.  Every cv2.resize of that block is s2v_resize_linear (INTER_LINEAR restated), the
pyramids are s2v_laplacian_blend, the mask is s2v_parse_mask.  There is no CPU path: CPU torch
tensors raise and a missing libs2v.so raises.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from ._lib import check
from .ops import NHWC

MASK_COLORMAP = [0] * 10 + [255, 255, 255] + [0] * 6          # face_parsing.py:30 (process_tensor)
PROCESS_MM = [0] + [255] * 12 + [0] * 6                        # face_parsing.py:39 (process default)
MOUTH_MM = [0] * 10 + [255, 255, 255] + [0] * 6                # inference.py:304

RS_U8, RS_F32, RS_F32_TO_U8, RS_U8_EQ255, RS_F64 = range(5)
_RS_IN = {RS_U8: torch.uint8, RS_F32: torch.float32, RS_F32_TO_U8: torch.float32, RS_U8_EQ255: torch.uint8,
          RS_F64: torch.float64}
_RS_OUT = {RS_U8: torch.uint8, RS_F32: torch.float32, RS_F32_TO_U8: torch.uint8, RS_U8_EQ255: torch.float32,
           RS_F64: torch.float64}

_CTX = {}


def _ctx(device) -> ops.Ctx:
    key = str(torch.device(device))
    if key not in _CTX:
        _CTX[key] = ops.Ctx(device)
    return _CTX[key]


def to_device(x, device="cuda") -> torch.Tensor:
    """NumPy array -> device tensor (a copy); device tensors pass through; CPU tensors raise."""
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x)).to(device)
    if not (isinstance(x, torch.Tensor) and x.is_cuda):
        raise RuntimeError("s2v_amd.post runs on the HIP device only: pass NumPy arrays or CUDA tensors "
                           "(there is no CPU fallback on the product path)")
    return x


def _hwc(t: torch.Tensor):
    """(n, h, w, c, row pitch, image pitch) of a [H,W], [H,W,C] or [N,H,W,C] view with unit channel
    stride (row / image pitches may be those of a larger frame: ROI views)."""
    if t.dim() == 2:
        t = t.unsqueeze(-1)
    if t.dim() == 3:
        t = t.unsqueeze(0)
    n, h, w, c = t.shape
    sn, sh, sw, sc = t.stride()
    if sc != 1 or sw != c:
        raise ValueError("resize_linear: pixels must be packed (channel stride 1, pixel stride C)")
    return n, h, w, c, sh, sn


def resize_linear(x: torch.Tensor, dsize, out: torch.Tensor | None = None, mode: int | None = None, fxfy=None):
    """cv2.resize(x, dsize=(W, H), interpolation=INTER_LINEAR) on a device image ([H,W], [H,W,C] or a
    batch [N,H,W,C], uint8, float32 or float64).  ``out`` may be a view into a larger frame.  mode
    (default by dtype): RS_U8, RS_F32, RS_F32_TO_U8 (np.uint8 of the float result), RS_U8_EQ255
    (1.0 where the resized uint8 value is 255, else 0), RS_F64.  ``fxfy``: cv2.resize(x, (0, 0),
    fx, fy) (dsize must then be (round(w fx), round(h fy)); the factors themselves scale)."""
    W, H = dsize
    if mode is None:
        mode = {torch.uint8: RS_U8, torch.float64: RS_F64}.get(x.dtype, RS_F32)
    if x.dtype != _RS_IN[mode]:
        raise TypeError(f"resize_linear: mode {mode} does not take {x.dtype}")
    n, h, w, c, xrs, xis = _hwc(x)
    odt = _RS_OUT[mode]
    if out is None:
        shape = {2: (H, W), 3: (H, W, c)}.get(x.dim(), (n, H, W, c))
        out = torch.empty(shape, dtype=odt, device=x.device)
    on, oh, ow, oc, yrs, yis = _hwc(out)
    if (on, oh, ow, oc) != (n, H, W, c) or out.dtype != odt:
        raise ValueError(f"resize_linear: out {tuple(out.shape)} {out.dtype} != {(n, H, W, c)} {odt}")
    ctx = _ctx(x.device)
    if fxfy is not None:
        check(ctx.lib.s2v_resize_linear_fxfy(x.data_ptr(), n, h, w, c, xrs, xis, out.data_ptr(), H, W, yrs, yis, mode,
                                             float(fxfy[0]), float(fxfy[1]), ctx.stream), "s2v_resize_linear_fxfy")
        return out
    check(ctx.lib.s2v_resize_linear(x.data_ptr(), n, h, w, c, xrs, xis, out.data_ptr(), H, W, yrs, yis, mode,
                                    ctx.stream), "s2v_resize_linear")
    return out


def laplacian_pyramid_blending_with_mask(A, B, m, num_levels=6, clip=False):
    """futils/inference_utils.py:181-222 on the device: A, B uint8 [H,W,C] (or [N,H,W,C]), m fp32
    [H,W] (or [N,H,W]) -> fp32 blended image; ``clip`` fuses the caller's np.clip(., 0, 255)."""
    dev = A.device if isinstance(A, torch.Tensor) else "cuda"
    A, B = to_device(A, dev).contiguous(), to_device(B, dev).contiguous()
    m = to_device(m, dev).float().contiguous()
    if A.dtype != torch.uint8 or B.dtype != torch.uint8:
        raise TypeError("laplacian_pyramid_blending_with_mask: A and B are uint8 images (cv2 frames)")
    n, h, w, c, _, _ = _hwc(A)
    if B.shape != A.shape or m.numel() != n * h * w:
        raise ValueError("laplacian_pyramid_blending_with_mask: A, B, m shapes disagree")
    ctx = _ctx(dev)
    out = torch.empty(A.shape, dtype=torch.float32, device=dev)
    need = ctx.lib.s2v_laplacian_blend_ws_bytes(n, h, w, c, num_levels)
    ws, wsb = ctx.ws.get(need)
    check(ctx.lib.s2v_laplacian_blend(A.data_ptr(), B.data_ptr(), m.data_ptr(), n, h, w, c, num_levels, int(clip),
                                      out.data_ptr(), ws, wsb, ctx.stream), "s2v_laplacian_blend")
    return out


_CMAPS = {}


def _cmap(colormap, device) -> torch.Tensor:
    """Device copy of a colormap, made once (not inside a graph capture)."""
    key = (tuple(int(v) for v in colormap), str(device))
    if key not in _CMAPS:
        _CMAPS[key] = torch.tensor(key[0], dtype=torch.uint8).to(device)
    return _CMAPS[key]


def parse_mask(logits: NHWC, colormap, out: torch.Tensor | None = None) -> torch.Tensor:
    """argmax over the parsing channels of NHWC logits -> colormap value, uint8 [N,H,W]."""
    ctx = _ctx(logits.t.device)
    cmap = _cmap(colormap, logits.t.device)
    if out is None:
        out = torch.empty((logits.n, logits.h, logits.w), dtype=torch.uint8, device=logits.t.device)
    check(ctx.lib.s2v_parse_mask(logits.ptr, logits.n, logits.h, logits.w, logits.c, logits.h * logits.w * logits.cs,
                                 logits.cs, 1, cmap.data_ptr(), out.data_ptr(), None, ctx.stream), "s2v_parse_mask")
    return out


class FaceParse:
    """third_part/GPEN/face_parse/face_parsing.py:12-81 on the device.  ``net`` is an
    s2v_amd.models.ParseNet; without it the weights load from base_dir/weights/<model>.pth."""

    def __init__(self, base_dir="./", model="ParseNet-latest", device="cuda", net=None):
        import os
        from . import models
        self.size = 512
        self.device = torch.device(device)
        self.MASK_COLORMAP = list(MASK_COLORMAP)
        if net is None:
            net = models.load_parsenet(os.path.join(base_dir, "weights", model + ".pth"), self.size)
        self.faceparse = net.eval()

    def _engine(self):
        return self.faceparse._engine(self.device)

    def img2tensor_nhwc(self, im_u8: torch.Tensor) -> NHWC:
        """img2tensor (:59-63) into the engine's NHWC 4-channel layout; im_u8 [H,W,3] or [N,H,W,3] BGR."""
        _, ctx = self._engine()
        n, h, w, _, _, _ = _hwc(im_u8)
        x4 = NHWC.empty(n, h, w, 4, self.device)
        check(ctx.lib.s2v_img_u8_to_m11(im_u8.contiguous().data_ptr(), n * h * w, 1, x4.ptr, 4, ctx.stream),
              "s2v_img_u8_to_m11")
        return x4

    def masks_device(self, im_u8_512: torch.Tensor, mm=PROCESS_MM) -> torch.Tensor:
        """[N,512,512,3] (or [512,512,3]) uint8 BGR device images -> uint8 masks [N,512,512]."""
        eng, ctx = self._engine()
        logits = eng.mask_logits(ctx, self.img2tensor_nhwc(im_u8_512))
        return parse_mask(logits, mm)

    def process(self, im, mm=PROCESS_MM):
        """face_parsing.py:39-45: cv2.resize to 512, img2tensor, ParseNet, tenor2mask -> [uint8 512x512]
        (NumPy, like the reference's list of masks)."""
        im = to_device(im, self.device)
        im512 = resize_linear(im, (self.size, self.size))
        return [m.cpu().numpy() for m in self.masks_device(im512, mm)]

    def process_tensor(self, imt):
        """face_parsing.py:47-57: imt [B,3,H,W] in [0,1] RGB -> nearest resize of flip(1)*2-1 to 512 ->
        argmax -> MASK_COLORMAP, returned as int64 [1,B,512,512] like the reference."""
        eng, ctx = self._engine()
        imt = to_device(imt, self.device).float()
        b, _, h, w = imt.shape
        x4 = NHWC.empty(b, self.size, self.size, 4, self.device)
        ops.fill(ctx, x4.t)
        sn, sc, sy, sx = imt.stride()                           # flip(1): channel 2 first, stride -sc
        ops.resize(ctx, imt, 2 * sc, (b, 3, h, w), (sn, -sc, sy, sx), x4.t, 0,
                   (self.size, self.size), ops.nhwc_strides(x4.slice(0, 3)), mode=1)
        ops.eltwise(ctx, x4.slice(0, 3), x4.slice(0, 3), a=2.0, bias=torch.full((3,), -1.0, device=self.device))
        m = parse_mask(eng.mask_logits(ctx, x4), self.MASK_COLORMAP)
        return m.long().unsqueeze(0)


class MouthBlend:
    """inference.py:302-313 given GFPGAN's restored frame: FaceParse mouth mask of the face box, the
    binary mask pasted into the frame (:305-308), the three 512x512 resizes, the 10-level Laplacian
    blend, np.clip and the uint8 resize back (:310-313).  Frames are uint8 HWC BGR."""

    def __init__(self, parser: FaceParse, levels: int = 10, mm=MOUTH_MM):
        self.parser, self.levels, self.mm = parser, levels, list(mm)

    def run(self, restored, ff, coords, out: torch.Tensor | None = None) -> torch.Tensor:
        return self.run_batch([restored], [ff], [coords], None if out is None else out[None])[0]

    def run_batch(self, restored, ff, coords, out: torch.Tensor | None = None) -> torch.Tensor:
        """restored, ff: [N,H,W,3] uint8 device tensors (or lists of [H,W,3]); coords: N boxes
        (y1, y2, x1, x2) -> [N,H,W,3] uint8."""
        dev = self.parser.device
        R = torch.stack([to_device(r, dev) for r in restored]) if isinstance(restored, (list, tuple)) \
            else to_device(restored, dev)
        Fr = torch.stack([to_device(f, dev) for f in ff]) if isinstance(ff, (list, tuple)) else to_device(ff, dev)
        n, H, W, _ = R.shape
        S = self.parser.size
        crops = torch.empty((n, S, S, 3), dtype=torch.uint8, device=dev)
        for i, (y1, y2, x1, x2) in enumerate(coords):
            resize_linear(R[i, y1:y2, x1:x2], (S, S), out=crops[i])
        tmp = self.parser.masks_device(crops, self.mm)              # [N,512,512] uint8
        return self.compose(R, Fr, tmp, coords, out)

    def compose(self, R: torch.Tensor, Fr: torch.Tensor, tmp: torch.Tensor, coords, out=None) -> torch.Tensor:
        """Everything after the parse (inference.py:306-313) given the uint8 512x512 masks ``tmp``."""
        dev = R.device
        n, H, W, _ = R.shape
        S = self.parser.size
        full = torch.empty((n, H, W), dtype=torch.float32, device=dev)
        ops.fill(_ctx(dev), full)
        for i, (y1, y2, x1, x2) in enumerate(coords):
            resize_linear(tmp[i], (x2 - x1, y2 - y1), out=full[i, y1:y2, x1:x2], mode=RS_U8_EQ255)
        A, B = resize_linear(R, (S, S)), resize_linear(Fr, (S, S))
        M = resize_linear(full.unsqueeze(-1), (S, S)).squeeze(-1)
        img = laplacian_pyramid_blending_with_mask(A, B, M, self.levels, clip=True)
        if out is None:
            out = torch.empty((n, H, W, 3), dtype=torch.uint8, device=dev)
        return resize_linear(img, (W, H), out=out, mode=RS_F32_TO_U8)
