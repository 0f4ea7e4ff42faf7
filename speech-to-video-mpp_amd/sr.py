"""Frame super-resolution on the device: RealESRNet
(third_part/GPEN/sr_model/real_esrnet.py), the `enhancer.srmodel.process(img)` call that
FaceEnhancement.process makes on every full frame (face_enhancement.py:102-105; inference.py:228-231
builds it with sr_scale=2, sr_model=None -> weights/realesrnet_x2.pth, num_feat=32).

    from s2v_amd.sr import RealESRNet
    sr = RealESRNet("checkpoints", None, scale=2)     # real_esrnet.py:8-19
    big = sr.process(frame_u8_bgr)                    # [H,W,3] uint8 -> [2H,2W,3] uint8

The uint8 -> float / reflect-pad front end is s2v_sr_u8_in, the clamp / round / BGR back end is
s2v_sr_f32_out, the net is models.RRDBNet (engine/rrdb.py).  Same constructor, ``tile_process``
bookkeeping and error behaviour as the reference: ``process`` prints 'sr failed: ...' and returns
None on a failure inside the forward.  There is no CPU path: CPU torch tensors raise, and a missing
libs2v.so raises at construction.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import models
from ._lib import check
from .ops import NHWC


class RealESRNet:
    """real_esrnet.py:8-137."""

    def __init__(self, base_dir="./", model=None, scale=2, tile_size=0, tile_pad=10, num_feat=32, device="cuda",
                 net=None):
        self.base_dir = base_dir
        self.scale = scale
        self.tile_size = tile_size
        self.tile_pad = tile_pad
        self.device = torch.device(device)
        self.num_feat = num_feat
        self.model = model
        if net is None:
            self.load_srmodel(base_dir, model)
        else:
            self.srmodel = net.eval()
        self.eng, self.ctx = self.srmodel._engine(self.device)

    def load_srmodel(self, base_dir, model):
        """real_esrnet.py:21-30."""
        name = "realesrnet_x%d.pth" % self.scale if model is None else model + "_x%d.pth" % self.scale
        self.srmodel = models.load_srmodel(os.path.join(base_dir, "weights", name), self.scale, self.num_feat)

    @property
    def mod_scale(self):
        return {2: 2, 1: 4}.get(self.scale)

    # ------------------------------------------------------------------ device pieces
    def to_input(self, frames_u8: torch.Tensor) -> tuple[NHWC, int, int]:
        """[N,H,W,3] uint8 BGR device frames -> (x / 255 RGB, reflect-padded 4-channel NHWC, h_pad,
        w_pad) (real_esrnet.py:100-115)."""
        n, h, w, c = frames_u8.shape
        assert c == 3 and frames_u8.dtype == torch.uint8
        m = self.mod_scale
        h_pad = (m - h % m) if m and h % m else 0
        w_pad = (m - w % m) if m and w % m else 0
        x4 = NHWC.empty(n, h + h_pad, w + w_pad, 4, self.device)
        check(self.ctx.lib.s2v_sr_u8_in(frames_u8.contiguous().data_ptr(), n, h, w, 1, h_pad, w_pad, x4.ptr, 4,
                                        self.ctx.stream), "s2v_sr_u8_in")
        return x4, h_pad, w_pad

    def to_u8(self, y: NHWC, h: int, w: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """Crop / clamp / round / RGB -> BGR (real_esrnet.py:125-131) -> [N,h,w,3] uint8."""
        if out is None:
            out = torch.empty((y.n, h, w, 3), dtype=torch.uint8, device=self.device)
        check(self.ctx.lib.s2v_sr_f32_out(y.ptr, y.n, h, w, y.h, y.w, y.cs, 1, out.data_ptr(), self.ctx.stream),
              "s2v_sr_f32_out")
        return out

    def upscale_nhwc(self, x4: NHWC) -> NHWC:
        s = self.scale
        y = NHWC.empty(x4.n, x4.h * s, x4.w * s, 3, self.device)
        return self.eng.forward_nhwc(self.ctx, x4, y)

    def tile_process(self, x4: NHWC) -> NHWC:
        """real_esrnet.py:34-97 on the NHWC input: each padded tile runs the net on its own, the
        unpadded part of its output is placed in the full output."""
        n, height, width = x4.n, x4.h, x4.w
        s, ts, tp = self.scale, self.tile_size, self.tile_pad
        out = NHWC.empty(n, height * s, width * s, 3, self.device)
        for ty in range(math.ceil(height / ts)):
            for tx in range(math.ceil(width / ts)):
                sx, sy = tx * ts, ty * ts
                ex, ey = min(sx + ts, width), min(sy + ts, height)
                sxp, exp_ = max(sx - tp, 0), min(ex + tp, width)
                syp, eyp = max(sy - tp, 0), min(ey + tp, height)
                tile = NHWC(x4.t[:, syp:eyp, sxp:exp_, :].contiguous())
                t_out = self.upscale_nhwc(tile)
                ox, oy = (sx - sxp) * s, (sy - syp) * s
                out.t[:, sy * s:ey * s, sx * s:ex * s, :] = \
                    t_out.t[:, oy:oy + (ey - sy) * s, ox:ox + (ex - sx) * s, :]
        return out

    def process_device(self, frames_u8: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """[N,H,W,3] (or [H,W,3]) uint8 BGR device frames -> [N,sH',sW',3] uint8 BGR device frames
        (sH' = s H for sizes that need no padding)."""
        single = frames_u8.dim() == 3
        if single:
            frames_u8 = frames_u8.unsqueeze(0)
        x4, h_pad, w_pad = self.to_input(frames_u8)
        y = self.tile_process(x4) if self.tile_size > 0 else self.upscale_nhwc(x4)
        # the reference removes only h_pad / w_pad rows / columns from the *upscaled* output
        # (real_esrnet.py:126-128): an odd 27x31 frame at x2 comes back 55x63
        res = self.to_u8(y, y.h - h_pad, y.w - w_pad, out)
        return res[0] if single else res

    @torch.no_grad()
    def process(self, img):
        """real_esrnet.py:99-137: one uint8 HWC BGR frame (NumPy or device tensor) -> uint8 HWC BGR
        NumPy array, or None (with the reference's message) if the forward fails."""
        if isinstance(img, np.ndarray):
            img = torch.from_numpy(np.ascontiguousarray(img)).to(self.device)
        elif not (isinstance(img, torch.Tensor) and img.is_cuda):
            raise RuntimeError("s2v_amd.sr runs on the HIP device only: pass a NumPy array or a CUDA tensor "
                               "(there is no CPU fallback on the product path)")
        try:
            return self.process_device(img).cpu().numpy()
        except Exception as e:  # noqa: BLE001 - the reference's contract (real_esrnet.py:136-137)
            print("sr failed:", e)
            return None
