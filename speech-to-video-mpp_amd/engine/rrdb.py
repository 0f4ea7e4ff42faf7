"""RRDBNet (RealESRNet) engine (third_part/GPEN/sr_model/rrdbnet_arch.py:8-116), NHWC on libs2v.

Layout and fusions:
  * pixel_unshuffle (arch_util.py:106-125) is folded into conv_first: a 3x3 conv over the
    r x r unshuffled channels c*r^2 + i*r + j equals a (3r)x(3r), stride-r, pad-r conv of the
    image itself with W'[o, c, ty, tx] = W[o, c*r^2 + (ty % r)*r + tx % r, ty // r, tx // r],
    so no unshuffled copy is ever written;
  * the dense concatenations torch.cat((x, x1, .., x4), 1) of every ResidualDenseBlock
    (:30-37) are channel ranges of one [B, h, w, nf + 4 g] buffer: conv_i reads the prefix
    [0, nf + (i-1) g) and writes its g channels right after it (bias + lrelu(0.2) fused);
  * conv5's `x5 * 0.2 + x` is its epilogue (scale 0.2 folded into the weights' scale/shift,
    residual x) and it writes the next block's input slice directly;
  * RRDB's `out * 0.2 + x` (:56-61) is one elementwise pass (eltwise) into the first buffer;
  * the two nearest x2 upsamplings (:111-112) are the conv's IN_NEAREST_UP2 gather mode;
  * `feat + conv_body(body)` is conv_body's residual epilogue.
"""
from __future__ import annotations

import torch

from .. import ops
from ..ops import NHWC, ConvW

LRELU = 0.2


def _unshuffle_weight(w: torch.Tensor, r: int, cin: int) -> torch.Tensor:
    """[O, cin*r*r, 3, 3] conv over pixel_unshuffle(x, r) -> [O, cin, 3r, 3r] conv over x."""
    o = w.shape[0]
    w = w.reshape(o, cin, r, r, 3, 3)                  # [o, c, i, j, ky, kx]
    return w.permute(0, 1, 4, 2, 5, 3).reshape(o, cin, 3 * r, 3 * r)   # ty = ky*r + i, tx = kx*r + j


class RRDBEngine:
    def __init__(self, sd, device, scale: int, num_in_ch=3):
        dev = torch.device(device)
        self.device, self.scale = dev, scale
        self.r = {4: 1, 2: 2, 1: 4}[scale]
        self.num_block = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("body."))
        f = lambda p: sd[p + "weight"].float()  # noqa: E731
        b = lambda p: sd[p + "bias"].float()    # noqa: E731
        self.nf = sd["conv_first.weight"].shape[0]
        self.g = sd["body.0.rdb1.conv1.weight"].shape[0]
        self.cin = num_in_ch
        self.cin_pad = 4 if num_in_ch == 3 else num_in_ch
        wf = _unshuffle_weight(f("conv_first."), self.r, num_in_ch) if self.r > 1 else f("conv_first.")
        self.conv_first = ConvW(ops.pad_cin(wf, self.cin_pad), b("conv_first."), dev, stride=self.r,
                                padding=self.r)
        self.blocks = []
        for i in range(self.num_block):
            rdbs = []
            for r in (1, 2, 3):
                p = f"body.{i}.rdb{r}."
                convs = [ConvW(f(f"{p}conv{k}."), b(f"{p}conv{k}."), dev, padding=1) for k in range(1, 5)]
                convs.append(ConvW(f(p + "conv5."), b(p + "conv5."), dev, padding=1, post_scale=0.2))
                rdbs.append(convs)
            self.blocks.append(rdbs)
        self.conv_body = ConvW(f("conv_body."), b("conv_body."), dev, padding=1)
        self.conv_up1 = ConvW(f("conv_up1."), b("conv_up1."), dev, padding=1, in_mode=ops.IN_NEAREST_UP2)
        self.conv_up2 = ConvW(f("conv_up2."), b("conv_up2."), dev, padding=1, in_mode=ops.IN_NEAREST_UP2)
        self.conv_hr = ConvW(f("conv_hr."), b("conv_hr."), dev, padding=1)
        self.conv_last = ConvW(f("conv_last."), b("conv_last."), dev, padding=1)
        self.cout = self.conv_last.cout

    def out_hw(self, h, w):
        return h * self.scale, w * self.scale

    def _rdb(self, ctx, convs, buf: NHWC, dst: NHWC):
        nf, g = self.nf, self.g
        for k in range(4):
            ops.conv2d(ctx, buf.slice(0, nf + k * g), convs[k], buf.slice(nf + k * g, g),
                       act=ops.ACT_LRELU, alpha=LRELU)
        ops.conv2d(ctx, buf.slice(0, nf + 4 * g), convs[4], dst, res=buf.slice(0, nf))

    def forward_nhwc(self, ctx, x: NHWC, y: NHWC):
        """x: NHWC [B, H, W, >=3 (4-padded)] view with H, W multiples of the unshuffle factor ->
        y: NHWC [B, scale H, scale W, num_out_ch] view (written)."""
        dev, nf, g = self.device, self.nf, self.g
        n = x.n
        assert x.c == self.cin_pad, f"RRDBNet engine: input view has {x.c} channels, expects {self.cin_pad}"
        assert x.h % self.r == 0 and x.w % self.r == 0, "RRDBNet: input size must be a multiple of the unshuffle factor"
        h, w = x.h // self.r, x.w // self.r
        ct = nf + 4 * g
        bufs = [NHWC.empty(n, h, w, ct, dev) for _ in range(3)]
        feat = NHWC.empty(n, h, w, nf, dev)
        ops.conv2d(ctx, x, self.conv_first, feat)
        ops.eltwise(ctx, feat, bufs[0].slice(0, nf))
        a, b_, c = bufs
        for rdbs in self.blocks:
            self._rdb(ctx, rdbs[0], a, b_.slice(0, nf))
            self._rdb(ctx, rdbs[1], b_, c.slice(0, nf))
            self._rdb(ctx, rdbs[2], c, b_.slice(0, nf))
            ops.eltwise(ctx, b_.slice(0, nf), a.slice(0, nf), a=0.2, add=a.slice(0, nf))
        body = NHWC.empty(n, h, w, nf, dev)
        ops.conv2d(ctx, a.slice(0, nf), self.conv_body, body, res=feat)
        del bufs, a, b_, c
        u1 = NHWC.empty(n, 2 * h, 2 * w, nf, dev)
        ops.conv2d(ctx, body, self.conv_up1, u1, act=ops.ACT_LRELU, alpha=LRELU)
        u2 = NHWC.empty(n, 4 * h, 4 * w, nf, dev)
        ops.conv2d(ctx, u1, self.conv_up2, u2, act=ops.ACT_LRELU, alpha=LRELU)
        hr = NHWC.empty(n, 4 * h, 4 * w, nf, dev)
        ops.conv2d(ctx, u2, self.conv_hr, hr, act=ops.ACT_LRELU, alpha=LRELU)
        ops.conv2d(ctx, hr, self.conv_last, y)
        return y

    def forward(self, ctx, x: torch.Tensor, out: torch.Tensor):
        """x [B, C, H, W] NCHW device tensor -> out [B, C_out, scale H, scale W] (written)."""
        n, c, hh, ww = x.shape
        assert c == self.cin, f"RRDBNet engine built for {self.cin} input channels"
        x4 = NHWC.empty(n, hh, ww, self.cin_pad, self.device)
        if self.cin_pad != c:
            ops.fill(ctx, x4.t)
        ops.nchw_to_nhwc(ctx, x, x4.slice(0, c))
        oh, ow = self.out_hw(hh, ww)
        y = NHWC.empty(n, oh, ow, self.cout, self.device)
        self.forward_nhwc(ctx, x4, y)
        ops.nhwc_to_nchw(ctx, y, out)
        return out
