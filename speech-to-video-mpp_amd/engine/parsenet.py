"""ParseNet engine (third_part/GPEN/face_parse/parse_model.py:69-75, blocks.py:72-126), NHWC on libs2v.

Every ConvLayer is one s2v_conv2d launch: ReflectionPad2d is the conv's reflect addressing
(S2V_PAD_REFLECT), scale='up' (nearest x2) is the IN_NEAREST_UP2 gather reflected in the upsampled
frame, 'down' is stride 2, eval BatchNorm folds into the epilogue scale/shift and the activation
runs in the epilogue.  A ResidualBlock's sum (identity + conv2(conv1(x))) is conv2's epilogue
residual; the body skip (feat + body(feat), :71) is one elementwise add.  The mask head and the
image head read the same decoder output; the mask-only path (FaceParse) skips the image head.
"""
from __future__ import annotations

import torch

from .. import ops
from ..ops import NHWC, ConvW

ACTS = {"relu": (ops.ACT_RELU, 0.0), "leakyrelu": (ops.ACT_LRELU, 0.2), "none": (ops.ACT_NONE, 0.0)}


class _Layer:
    def __init__(self, sd, p, spec, dev, cin_pad=0):
        if spec["relu"] not in ACTS:
            raise NotImplementedError(f"ParseNet engine: activation {spec['relu']!r} (FaceParse uses LeakyReLU)")
        if spec["norm"] not in ("bn", "none"):
            raise NotImplementedError(f"ParseNet engine: norm {spec['norm']!r} (FaceParse uses eval BatchNorm)")
        w = sd[p + "conv2d.weight"].float()
        if cin_pad:
            w = ops.pad_cin(w, cin_pad)
        bn = None
        if spec["norm"] == "bn":
            q = p + "norm.norm."
            bn = (sd[q + "weight"], sd[q + "bias"], sd[q + "running_mean"], sd[q + "running_var"])
        self.cw = ConvW(w, sd.get(p + "conv2d.bias"), dev, stride=2 if spec["scale"] == "down" else 1,
                        padding=spec["pad"], pad_mode=ops.PAD_REFLECT,
                        in_mode=ops.IN_NEAREST_UP2 if spec["scale"] == "up" else ops.IN_DIRECT, bn=bn)
        self.act, self.alpha = ACTS[spec["relu"]]

    def __call__(self, ctx, x: NHWC, res: NHWC | None = None, out: NHWC | None = None) -> NHWC:
        oh, ow = self.cw.out_hw(x.h, x.w)
        y = out if out is not None else NHWC.empty(x.n, oh, ow, self.cw.cout, x.t.device)
        ops.conv2d(ctx, x, self.cw, y, act=self.act, alpha=self.alpha, res=res, res_after=res is not None)
        return y


class ParseNetEngine:
    def __init__(self, sd, device, desc):
        dev = torch.device(device)
        self.device = dev
        self.enc0 = _Layer(sd, desc["enc0"][0], desc["enc0"][1], dev, cin_pad=4)

        def block(b):
            p, sc, c1, c2 = b
            return (None if sc is None else _Layer(sd, p + "shortcut_func.", sc, dev),
                    _Layer(sd, p + "conv1.", c1, dev), _Layer(sd, p + "conv2.", c2, dev))
        self.down = [block(b) for b in desc["down"]]
        self.body = [block(b) for b in desc["body"]]
        self.up = [block(b) for b in desc["up"]]
        self.out_img = _Layer(sd, desc["out_img"][0], desc["out_img"][1], dev)
        self.out_mask = _Layer(sd, desc["out_mask"][0], desc["out_mask"][1], dev)

    @staticmethod
    def _res(ctx, blk, x: NHWC) -> NHWC:
        sc, c1, c2 = blk
        ident = x if sc is None else sc(ctx, x)
        return c2(ctx, c1(ctx, x), res=ident)

    def features(self, ctx, x4: NHWC) -> NHWC:
        """x4: NHWC [B,H,W,4] image in [-1,1] (channel 3 zero) -> decoder output (parse_model.py:70-72)."""
        f = self.enc0(ctx, x4)
        for blk in self.down:
            f = self._res(ctx, blk, f)
        h = f
        for blk in self.body:
            h = self._res(ctx, blk, h)
        s = NHWC.empty(f.n, f.h, f.w, f.c, self.device)
        ops.eltwise(ctx, f, s, add=h)                           # feat + body(feat)
        for blk in self.up:
            s = self._res(ctx, blk, s)
        return s

    def mask_logits(self, ctx, x4: NHWC) -> NHWC:
        return self.out_mask(ctx, self.features(ctx, x4))

    def forward(self, ctx, x: torch.Tensor, mask_out: torch.Tensor, img_out: torch.Tensor | None):
        """x [B,3,H,W] NCHW device tensor -> out_mask [B,19,H,W], out_img [B,3,H,W] (written)."""
        b, _, H, W = x.shape
        x4 = NHWC.empty(b, H, W, 4, self.device)
        ops.fill(ctx, x4.t)
        ops.nchw_to_nhwc(ctx, x, x4.slice(0, 3))
        d = self.features(ctx, x4)
        ops.nhwc_to_nchw(ctx, self.out_mask(ctx, d), mask_out)
        if img_out is not None:
            ops.nhwc_to_nchw(ctx, self.out_img(ctx, d), img_out)
        return mask_out, img_out
