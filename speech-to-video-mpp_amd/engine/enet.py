"""ENet engine (reference models/ENet.py:82-139): style encoder + LNet + two StyleGAN2 stages.

Modulated convolutions (base_blocks.py:460-554): the per-sample weights W * s[b, i] * demod[b, o]
(demod = rsqrt(sum_i s_i^2 sum_k W_oik^2 + eps), times sqrt(2)) are materialised by one small
kernel (s2v_modulate_weights, a few MB per layer) and the conv runs in batch mode with them, so
the implicit GEMM carries no prologue / epilogue scaling; noise and bias stay in the epilogue.
(The engine can also run them as conv(x * s, W) * demod with shared weights: ops.conv2d's
in_scale / nc_scale, used where per-sample weights do not apply.)
"""
from __future__ import annotations

import math
import os

import torch

from .. import ops
from ..ops import NHWC, ConvW
from .lnet import LNetEngine

LRELU = 0.2  # ENet.py:94-97, base_blocks.py:41-44, :522
# the style encoder and LNet are independent until the StyleConvs (ENet.py:94-112): run the style
# encoder on a side stream beside LNet (S2V_ENET_OVERLAP=0 serialises them)
OVERLAP = os.environ.get("S2V_ENET_OVERLAP", "1") == "1"
# ToRGB and its skip upsample as one pass (ops.torgb_up2); S2V_ENET_FUSED_TORGB=0: resize + small conv
FUSED_TORGB = os.environ.get("S2V_ENET_FUSED_TORGB", "1") == "1"
# x2-upsample StyleConvs on >= 32 channels as one polyphase conv over the un-upsampled input
# (ops.modulated_conv2d d2s: the bilinear taps folded into 4 parity-class filters, written depth-to-space)
# plus the four border lines recomputed exactly; S2V_ENET_POLY_UP=0: upsample pass + conv
POLY_UP = os.environ.get("S2V_ENET_POLY_UP", "1") == "1"
# the first StyleConv (the 4-channel RGB input carried as 4, 100^2 -> 200^2) polyphase too: its K = 36 gather
# then runs over the 100^2 input with the four parity classes as 4 x 256 output columns.  Measured slower on
# MI355X (r05, lipsync 24.6-24.7 vs 24.1-24.2 ms, profiles/r05_ab_lnet_pair.txt): off by default
POLY_UP4 = os.environ.get("S2V_ENET_POLY_UP4", "0") == "1"
# the style encoder's split-precision convs (launched beside LNet) as persistent blocks on half the
# device's CUs (s2v_conv_params.grid_cap, ops.half_chip_blocks): the CUs they leave free take LNet's
# latency-bound kernels as soon as they are launched instead of after the encoder's 100-200 us tiles
# drain.  On MI355X (256 CUs: 128 blocks, which divides every encoder layer's tile count), lipsync B=16
# 29.1 -> 26.1-26.5 ms (caps 192: 28.5, 160: 27.1, 112: 28.9, 96: 31.4, 64: 38.9; r03).
# S2V_ENET_STYLE_GRID: an explicit block count (0: one block per tile).
STYLE_GRID = os.environ.get("S2V_ENET_STYLE_GRID", "half")
# the first StyleConv (3x3 over the 4-channel RGB input carried as 4, after the x2 upsample) as a row-tap
# packed 3x1 conv (ConvW.make_rowpack + ops.row_pack: the (kx, c) taps become 12 of 32 packed channels) on
# the buffer-load tiles instead of the per-element gather of a 4-channel input; its modulation is the
# bank's segment laid out per packed channel (s'[kx * 4 + c] = s[c]).  Measured on MI355X (r06, same-box A/B,
# 3 pairs): lipsync 23.50 (gather) vs 23.59 ms (packed) -- off by default (S2V_ENET_ROWPACK0=1 turns it on)
ROWPACK0 = os.environ.get("S2V_ENET_ROWPACK0", "0") == "1"
# where the style-encoder branch forks off the calling stream: 0 = before LNet (both from the start of
# the step), h = before LNet's h x h decoder level (LNet's earlier levels then run on the whole chip)
FORK_AT = int(os.environ.get("S2V_ENET_FORK_AT", "0"))
# S2V_ENET_PAUSE="k:h": the style encoder runs its first conv and k down ResBlocks from the fork, then waits
# for LNet to reach its h x h decoder level (h = 0: LNet's end) and runs the rest from there, so the LNet
# levels in between (the latency-bound 12^2 FFC chain) have the whole chip.  Empty: no pause.
PAUSE = tuple(int(v) for v in os.environ.get("S2V_ENET_PAUSE", "").split(":")) if os.environ.get("S2V_ENET_PAUSE") else None
# S2V_ENET_PREMOD=1: the tail's StyleConv weights are modulated (W * s * d, ops.modulate_weights) on the style
# encoder's side stream right after the style code, beside LNet, instead of inside each StyleConv launch of the
# critical tail (the four polyphase edge strips then share one modulation)
PREMOD = os.environ.get("S2V_ENET_PREMOD", "1") == "1"
# S2V_ENET_STACK_STRIPS=1: the polyphase StyleConv's edge strips (the two outermost output lines per side) as one
# stacked strip image per axis: two upsample + conv launches instead of four
STACK_STRIPS = os.environ.get("S2V_ENET_STACK_STRIPS", "1") == "1"
# persistent blocks of the resumed part (S2V_ENET_RESUME_GRID; default: as STYLE_GRID)
RESUME_GRID = os.environ.get("S2V_ENET_RESUME_GRID", "")


def style_grid(device) -> int:
    """Persistent blocks of the style encoder's convs on ``device`` (STYLE_GRID)."""
    if STYLE_GRID == "half":
        return ops.half_chip_blocks(device)
    return int(STYLE_GRID)

# x2 bilinear upsample (align_corners=False) followed by a 3-tap conv, per output parity r: weight of
# input tap a (i-1, i, i+1) from conv tap p (-1, 0, 1), away from the image border
_FOLD = (((0.75, 0.25, 0.0), (0.25, 0.75, 0.75), (0.0, 0.0, 0.25)),
         ((0.25, 0.0, 0.0), (0.75, 0.75, 0.25), (0.0, 0.25, 0.75)))


def fold_up2_conv3(w: torch.Tensor) -> torch.Tensor:
    """[O, I, 3, 3] conv weights applied after a x2 bilinear upsample -> [4 O, I, 3, 3]: the 3x3 filters
    of the four output parity classes (ry, rx) (class-major) over the un-upsampled input."""
    f = torch.tensor(_FOLD, dtype=torch.float64)
    wd = w.double()
    return torch.cat([torch.einsum("ap,bq,oipq->oiab", f[ry], f[rx], wd) for ry in (0, 1) for rx in (0, 1)]).float()


class StyleLayer:
    """One ModulatedConv2d (StyleConv or ToRGB)."""

    def __init__(self, sd, p, device, demodulate, upsample, is_rgb):
        m = p + "modulated_conv."
        w = sd[m + "weight"].float()[0]                      # [O, I, k, k]
        self.k = w.shape[-1]
        if w.shape[1] == 3:                                  # 3-channel image input, carried as 4
            w = ops.pad_cin(w, 4)
        self.cin, self.cout = w.shape[1], w.shape[0]
        self.demodulate, self.upsample, self.is_rgb = demodulate, upsample, is_rgb
        bias = sd[p + "bias"].float().reshape(-1)
        self.conv = ConvW(w, bias, device, padding=self.k // 2)
        self.wsq = w.pow(2).sum((2, 3)).contiguous().to(device)   # [O, I]
        self.mod_w = sd[m + "modulation.weight"].float()
        self.mod_b = sd[m + "modulation.bias"].float()
        if self.mod_w.shape[0] < self.cin:                   # zero modulation for the padding channel
            self.mod_w = torch.cat([self.mod_w, torch.zeros(self.cin - self.mod_w.shape[0], self.mod_w.shape[1])])
            self.mod_b = torch.cat([self.mod_b, torch.zeros(self.cin - self.mod_b.shape[0])])
        self.noise_w = None if is_rgb else float(sd[p + "weight"].float().reshape(-1)[0])
        self.device = device
        self.conv4 = self.wsq4 = None
        if upsample and self.k == 3 and (self.cin % 32 == 0 or (POLY_UP4 and self.cin == 4)):
            self.conv4 = ConvW(fold_up2_conv3(w), bias.repeat(4), device, padding=1)
            self.wsq4 = self.wsq.repeat(4, 1).contiguous()
        self.rp = None                                       # row-packed form (ROWPACK0): packed channel count
        if ROWPACK0 and self.conv4 is None and not is_rgb and self.k == 3 and self.cin * self.k <= 32:
            self.conv.make_rowpack(device)
            self.rp = self.conv.rowpack.cin
            self.conv.rowpack.shift = self.conv.shift             # the layer bias in the packed conv's epilogue


class ENetEngine:
    def __init__(self, sd, device):
        dev = torch.device(device)
        self.device = dev
        self.lnet = LNetEngine(sd, dev, prefix="low_res.")
        # 3-channel images are carried as 4 channels (4th = 0) so their convs use the float4 gather
        self.first = ConvW(ops.pad_cin(sd["conv_body_first.weight"].float(), 4), sd["conv_body_first.bias"], dev)
        self.down = []
        for i in range(6):
            p = f"conv_body_down.{i}."
            # skip(interpolate(x, 0.5)) == a 2x2 stride-2 conv with the 1x1 weights / 4 on every tap
            # (bilinear x0.5 is the 2x2 mean and commutes with the 1x1 conv): no pooled copy of x
            sw = sd[p + "skip.weight"].float()
            skip2 = (sw / 4.0).expand(-1, -1, 2, 2).contiguous()
            self.down.append((ConvW(sd[p + "conv1.weight"], sd[p + "conv1.bias"], dev, padding=1),
                              ConvW(sd[p + "conv2.weight"], sd[p + "conv2.bias"], dev, padding=1),
                              ConvW(skip2, None, dev, stride=2)))
        self.final_conv = ConvW(sd["final_conv.weight"], sd["final_conv.bias"], dev, padding=1)
        # final_linear consumes feat.reshape(B, -1) in NCHW (c, h, w) order; our feature is NHWC
        # (h, w, c): permute the weight columns once.
        wl = sd["final_linear.weight"].float()
        c4 = sd["final_conv.weight"].shape[0]
        wl = wl.reshape(wl.shape[0], c4, 4, 4).permute(0, 2, 3, 1).reshape(wl.shape[0], -1)
        self.final_linear = ConvW(wl, sd["final_linear.bias"], dev)
        self.layers = []
        for i in range(2):
            self.layers.append(StyleLayer(sd, f"style_convs.{2 * i}.", dev, True, True, False))
            self.layers.append(StyleLayer(sd, f"style_convs.{2 * i + 1}.", dev, True, False, False))
            self.layers.append(StyleLayer(sd, f"to_rgbs.{i}.", dev, False, False, True))
        # all six modulation Linears consume the same style code -> one GEMM; each layer's segment
        # is padded to a multiple of 4 so the conv prologue can read s[n, c:c+4] as one 16-byte load
        offs, o, ws, bs = [], 0, [], []
        for l in self.layers:
            offs.append(o)
            mw, mb = l.mod_w, l.mod_b
            if l.rp is not None:
                # s'[kx * cin + c] = s[c] for kx < k, zero up to the packed width (ConvW.make_rowpack's channel
                # order); its first cin entries are s itself, which the demodulation reads
                z = l.rp - l.k * l.cin
                mw = torch.cat([mw] * l.k + [torch.zeros(z, mw.shape[1])])
                mb = torch.cat([mb] * l.k + [torch.zeros(z)])
            pad = (-mw.shape[0]) % 4
            ws += [mw, torch.zeros(pad, l.mod_w.shape[1])]
            bs += [mb, torch.zeros(pad)]
            o += mw.shape[0] + pad
        self.mod = ConvW(torch.cat(ws, 0), torch.cat(bs, 0), dev)
        self.mod_offs = offs
        self._demod = {}
        self.noise_seed = 0x5EED
        self.last_noises = [None] * 4

    def _side(self, ctx):
        """(stream, Ctx) of the calling lane for the style encoder branch (CUDA devices only)."""
        side = ctx.streams(("enet", id(self)), 1)
        return None if side is None else side[0]

    def _demod_table(self, poly):
        """The four StyleConvs' demodulations (base_blocks.py:492-494) as one ops.DemodRows table; a
        polyphase layer contributes its four parity-class blocks (wsq4)."""
        if poly not in self._demod:
            ls = [(self.mod_offs[j], self.layers[j].wsq4 if poly and self.layers[j].conv4 is not None
                   else self.layers[j].wsq) for j in (0, 1, 3, 4)]
            t = ops.DemodRows(ls, self.device)
            t.width = [w.shape[0] for _, w in ls]
            self._demod[poly] = t
        return self._demod[poly]

    def _demods(self, ctx, s2):
        """[B, nrows] demodulation vectors of the four StyleConvs, one launch (instead of one per layer
        in the tail): slot j of the table is columns [r0[j], + width[j])."""
        t = self._demod_table(POLY_UP)
        dall = ops.empty((s2.shape[0], t.nrows), self.device)
        ops.modconv_demod_rows(ctx, s2, t, dall, eps=1e-8, post=math.sqrt(2.0))
        return t, dall

    def _premodulate(self, ctx, s2, dtab, dall, b) -> dict:
        """PREMOD: the per-sample weights of the tail's StyleConvs, {layer index: {"conv4" / "conv": (wbuf,
        premod)}} (row-packed layers keep their in-launch modulation)."""
        wb = {}
        for st in range(2):
            for li in range(2):
                L, idx = self.layers[3 * st + li], 2 * st + li
                off = self.mod_offs[3 * st + li]
                r0, wd = dtab.r0[idx], dtab.width[idx]
                sv = s2[:, off: off + L.cin]
                if L.cin <= 4:
                    continue      # the 4-channel first StyleConv runs exact fp32 (conv_k4.hip): modulated in-launch
                if POLY_UP and L.conv4 is not None:
                    d4 = dall[:, r0: r0 + wd]
                    wb[idx] = {"conv4": ops.modulate_weights(ctx, L.conv4, sv, d4, b),
                               "conv": ops.modulate_weights(ctx, L.conv, sv, d4[:, : L.cout], b)}
                elif L.rp is None:
                    wb[idx] = {"conv": ops.modulate_weights(ctx, L.conv, sv, dall[:, r0: r0 + L.cout], b)}
        return wb

    def _poly_styleconv(self, ctx, L, cur: NHWC, s, d4, idx, noises, ctr, wb=None):
        """StyleConv(sample_mode='upsample') (base_blocks.py:500-533): F.interpolate(x, 2, bilinear) then
        the modulated 3x3 conv + noise + bias + LeakyReLU, as one depth-to-space conv over ``cur`` with
        the folded parity-class filters (L.conv4).  The fold assumes every upsampled row / column is an
        interior one: the clamped edge rows of the upsample and the conv's zero padding break that on
        the two outermost output lines of each side, so those are recomputed from 2-pixel strips of
        ``cur`` the direct way (upsample + conv with L.conv; every tap they read is exact) and copied
        in."""
        dev, b = self.device, cur.n
        h2, w2 = 2 * cur.h, 2 * cur.w
        d = d4[:, : L.cout]                                      # the class-0 block: the layer's own demod
        noise = None
        if L.noise_w:
            if noises is not None and noises[idx] is not None:
                noise = noises[idx].reshape(b, h2, w2).contiguous()
            else:
                noise = torch.empty((b, h2, w2), device=dev)
                ops.gaussian_noise(ctx, noise, self.noise_seed, idx << 36, ctr=ctr, shift=40)
                self.last_noises[idx] = noise
        y = NHWC.empty(b, h2, w2, L.cout, dev)
        kw = dict(act=ops.ACT_LRELU, alpha=LRELU, pix_w=L.noise_w or 0.0)
        wb = wb or {}
        ops.modulated_conv2d(ctx, cur, L.conv4, y, s, d4, pix_add=noise, d2s=True, premod=wb.get("conv4"), **kw)
        c = cur.c
        if STACK_STRIPS:
            # the two strips of one axis stacked into one 4-line image (first two lines | last two lines): one
            # upsample and one conv per axis instead of two.  The lines the kept outputs read never straddle the
            # seam: output lines 0, 1 read upsampled lines <= 2 (from source lines 0, 1 only) and 6, 7 read
            # lines >= 5 (source lines 2, 3 = the image's last two) or the conv's zero padding past line 7,
            # exactly as the separate strips do
            for axis, n_src, n_out in ((1, cur.h, h2), (2, cur.w, w2)):
                xs = NHWC(torch.cat([cur.t.narrow(axis, 0, 2), cur.t.narrow(axis, n_src - 2, 2)], axis))
                up = NHWC.empty(b, 2 * xs.h, 2 * xs.w, c, dev)
                ops.resize_nhwc(ctx, xs, up, scale_factor=2)
                ys = NHWC.empty(b, up.h, up.w, L.cout, dev)
                nz = None if noise is None else torch.cat([noise.narrow(axis, 0, 4), noise.narrow(axis, n_out - 4, 4)],
                                                          axis)
                ops.modulated_conv2d(ctx, up, L.conv, ys, s, d, pix_add=nz, premod=wb.get("conv"), **kw)
                y.t.narrow(axis, 0, 2).copy_(ys.t.narrow(axis, 0, 2))
                y.t.narrow(axis, n_out - 2, 2).copy_(ys.t.narrow(axis, 6, 2))
            return y
        # (x strip, its noise, the strip output lines kept, where they go): each strip's x2 upsample is
        # exact on the lines the kept outputs read (the clamped source row / column is the image's own)
        strips = ((cur.t[:, 0:2], lambda t: t[:, 0:4], lambda t: t[:, 0:2], lambda t: t[:, 0:2]),
                  (cur.t[:, cur.h - 2:], lambda t: t[:, h2 - 4:], lambda t: t[:, 2:4], lambda t: t[:, h2 - 2:]),
                  (cur.t[:, :, 0:2], lambda t: t[:, :, 0:4], lambda t: t[:, :, 0:2], lambda t: t[:, :, 0:2]),
                  (cur.t[:, :, cur.w - 2:], lambda t: t[:, :, w2 - 4:], lambda t: t[:, :, 2:4],
                   lambda t: t[:, :, w2 - 2:]))
        for xs_t, nsel, ssel, ysel in strips:
            xs = NHWC(xs_t.contiguous())
            up = NHWC.empty(b, 2 * xs.h, 2 * xs.w, c, dev)
            ops.resize_nhwc(ctx, xs, up, scale_factor=2)
            ys = NHWC.empty(b, up.h, up.w, L.cout, dev)
            nz = None if noise is None else nsel(noise).contiguous()
            ops.modulated_conv2d(ctx, up, L.conv, ys, s, d, pix_add=nz, premod=wb.get("conv"), **kw)
            ysel(y.t).copy_(ssel(ys.t))
        return y

    def style_code(self, ctx, ref: torch.Tensor):
        """ref: NCHW [B,3,H,W] device tensor -> style [B,1,1,512] (ENet.py:94-101)."""
        st = self.style_begin(ctx, ref)
        self.style_down(ctx, st, len(self.down))
        return self.style_end(ctx, st)

    def style_begin(self, ctx, ref: torch.Tensor) -> dict:
        """conv_body_first of the style encoder; returns the state style_down / style_end continue from."""
        dev, b = self.device, ref.shape[0]
        x = NHWC.empty(b, 256, 256, 4, dev)
        ops.fill(ctx, x.t)
        ops.nchw_to_nhwc(ctx, ref, x.slice(0, 3))                  # F.interpolate(ref, 256, bilinear)
        f = NHWC.empty(b, 256, 256, self.first.cout, dev)
        ops.conv2d(ctx, x, self.first, f, act=ops.ACT_LRELU, alpha=LRELU)
        return {"f": f, "i": 0}

    def style_down(self, ctx, st: dict, upto: int):
        """The down ResBlocks st["i"] .. upto - 1 (ResBlock(mode='down'), base_blocks.py:40-49)."""
        f, b, dev = st["f"], st["f"].n, self.device
        while st["i"] < min(upto, len(self.down)):
            c1, c2, sk = self.down[st["i"]]
            h, w = f.h, f.w
            td = NHWC.empty(b, h // 2, w // 2, c1.cout, dev)         # interpolate(lrelu(conv1(x)), 0.5):
            ops.conv2d(ctx, f, c1, td, act=ops.ACT_LRELU, alpha=LRELU, pool=True)   # pooled in the epilogue
            out = NHWC.empty(b, h // 2, w // 2, c2.cout, dev)
            ops.conv2d(ctx, f, sk, out)                             # skip(interpolate(x, 0.5))
            ops.conv2d(ctx, td, c2, out, act=ops.ACT_LRELU, alpha=LRELU, res=out, res_after=True)
            f = out
            st["i"] += 1
        st["f"] = f

    def style_end(self, ctx, st: dict):
        f, b, dev = st["f"], st["f"].n, self.device
        g = NHWC.empty(b, f.h, f.w, self.final_conv.cout, dev)
        ops.conv2d(ctx, f, self.final_conv, g, act=ops.ACT_LRELU, alpha=LRELU)
        style = NHWC.empty(b, 1, 1, self.final_linear.cout, dev)
        ops.conv2d(ctx, NHWC(g.t.view(b, 1, 1, -1)), self.final_linear, style)
        return style

    def forward(self, ctx, audio, face, gt, out: torch.Tensor, low: torch.Tensor, noises=None, aux=None):
        """audio [B,1,80,16], face [B,6,H,W], gt [B,3,H,W] (NCHW device tensors) ->
        out [B,3,384,384], low [B,3,96,96] (NCHW, written in place)."""
        dev = self.device
        b = audio.shape[0]
        svec = NHWC.empty(b, 1, 1, self.mod.cout, dev)
        side = self._side(ctx) if OVERLAP else None
        enc = {}

        def finish(sctx):
            enc["style"] = self.style_end(sctx, enc.pop("st"))
            ops.conv2d(sctx, enc["style"], self.mod, svec)
            enc["d"] = self._demods(sctx, svec.t.view(b, -1))       # off the tail: beside LNet
            if PREMOD:
                enc["wb"] = self._premodulate(sctx, svec.t.view(b, -1), enc["d"][0], enc["d"][1], b)

        def fork():
            sst, sctx = side
            sst.wait_stream(torch.cuda.current_stream(dev))
            with ops.x3_grid_cap(sctx, style_grid(dev)), ops.side_stream(sst, ctx.keep):
                enc["st"] = self.style_begin(sctx, face[:, 3:])
                self.style_down(sctx, enc["st"], PAUSE[0] if PAUSE else len(self.down))
                if not PAUSE:
                    finish(sctx)

        def resume():
            # the rest of the encoder after LNet's calling stream reached this point (stream order on the
            # side stream keeps it behind the first part)
            sst, sctx = side
            sst.wait_stream(torch.cuda.current_stream(dev))
            grid = int(RESUME_GRID) if RESUME_GRID else style_grid(dev)
            with ops.x3_grid_cap(sctx, grid), ops.side_stream(sst, ctx.keep):
                self.style_down(sctx, enc["st"], len(self.down))
                finish(sctx)

        on_level = None
        if side is not None:
            if FORK_AT:
                on_level = lambda h: fork() if h == FORK_AT and not enc else None  # noqa: E731
            else:
                fork()
                if PAUSE and PAUSE[1]:
                    on_level = lambda h: resume() if h == PAUSE[1] and "st" in enc else None  # noqa: E731
        else:
            enc["style"] = self.style_code(ctx, face[:, 3:])
            ops.conv2d(ctx, enc["style"], self.mod, svec)
            enc["d"] = self._demods(ctx, svec.t.view(b, -1))
        # LNet input: cat(inp, gt) -> bilinear 96x96 (ENet.py:103-104)
        x6 = NHWC.empty(b, 96, 96, 6, dev)
        ops.nchw_to_nhwc(ctx, face[:, :3], x6.slice(0, 3))
        ops.nchw_to_nhwc(ctx, gt, x6.slice(3, 3))
        lo = NHWC.empty(b, 96, 96, 4, dev)          # channel 3 = sigmoid(0): finite, zero weights
        self.lnet.forward(ctx, audio, x6, lo, pad_rgb=True, on_level=on_level)
        if side is not None and not enc:
            fork()                                             # FORK_AT names no LNet level
        if side is not None and "st" in enc:
            resume()                                           # PAUSE resumes at LNet's end
        ops.nhwc_to_nchw(ctx, lo.slice(0, 3), low)
        if side is not None:
            torch.cuda.current_stream(dev).wait_stream(side[0])    # style code ready for the StyleConvs
        style, (dtab, dall) = enc["style"], enc["d"]
        s2 = svec.t.view(b, -1)
        if aux is not None:
            aux["style"] = style.t.view(b, -1)
        # F.pad(reflect, 2) -> StyleConv / ToRGB stages (ENet.py:119-129)
        cur = NHWC.empty(b, 100, 100, 4, dev)
        ops.pad_reflect(ctx, lo, cur, (2, 2, 2, 2))
        skip = cur               # RGB + a finite pad channel: the x2 skip upsample takes the float4 path
        ctr = None
        # the noise planes drawn by this forward ([B, H, W] per StyleConv, None where the layer has no
        # noise or the caller passed it): kept referenced so that under a captured graph they stay
        # the buffers every replay draws into (tests compare a replay against the oracle with them)
        self.last_noises = [None] * 4
        if noises is None and any(L.noise_w for L in self.layers):
            ctr = ctx.noise(id(self)).bump(ctx)        # one draw per forward, also under graph replay
        for st in range(2):
            for li in range(2):
                L = self.layers[3 * st + li]
                off = self.mod_offs[3 * st + li]
                r0, wd = dtab.r0[2 * st + li], dtab.width[2 * st + li]
                if POLY_UP and L.conv4 is not None:
                    cur = self._poly_styleconv(ctx, L, cur, s2[:, off: off + L.cin], dall[:, r0: r0 + wd],
                                               2 * st + li, noises, ctr, wb=enc.get("wb", {}).get(2 * st + li))
                    continue
                x = cur
                if L.upsample:
                    x = NHWC.empty(b, 2 * cur.h, 2 * cur.w, cur.c, dev)
                    ops.resize_nhwc(ctx, cur, x, scale_factor=2)
                conv, cin = L.conv, L.cin
                if L.rp is not None:
                    xp = NHWC.empty(b, x.h, x.w, L.rp, dev)
                    ops.row_pack(ctx, x, xp, L.k, L.k // 2)
                    x, conv, cin = xp, L.conv.rowpack, L.rp
                d = dall[:, r0: r0 + L.cout]
                y = NHWC.empty(b, x.h, x.w, L.cout, dev)
                noise = None
                if L.noise_w:
                    if noises is not None and noises[2 * st + li] is not None:
                        noise = noises[2 * st + li].contiguous()
                    else:
                        noise = torch.empty((b, x.h, x.w), device=dev)
                        ops.gaussian_noise(ctx, noise, self.noise_seed, (2 * st + li) << 36, ctr=ctr, shift=40)
                        self.last_noises[2 * st + li] = noise
                pm = enc.get("wb", {}).get(2 * st + li, {}).get("conv") if L.rp is None else None
                ops.modulated_conv2d(ctx, x, conv, y, s2[:, off: off + cin], d, act=ops.ACT_LRELU, alpha=LRELU,
                                     pix_add=noise, pix_w=L.noise_w or 0.0, premod=pm)
                cur = y
            R = self.layers[3 * st + 2]
            off = self.mod_offs[3 * st + 2]
            rgb = NHWC.empty(b, cur.h, cur.w, 4, dev)
            if FUSED_TORGB and R.cin % 32 == 0 and (cur.h * cur.w) % 32 == 0:
                ops.torgb_up2(ctx, cur, R.conv, s2[:, off: off + R.cin], skip, rgb)   # + skip upsample (:552)
            else:
                ops.resize_nhwc(ctx, skip, rgb, scale_factor=2)      # skip upsample (base_blocks.py:552)
                ops.modulated_conv2d(ctx, cur, R.conv, rgb.slice(0, 3), s2[:, off: off + R.cin], res=rgb.slice(0, 3))
            skip = rgb
        ops.nhwc_to_nchw(ctx, skip.slice(0, 3), out, crop=(8, 8))    # [:, :, 8:-8, 8:-8]
        return out, low
