"""GFPGANv1Clean engine (third_part/GFPGAN/gfpgan/archs/gfpganv1_clean_arch.py:154-324 with the
StyleGAN2GeneratorCSFT decoder, stylegan2_clean_arch.py:185-367), NHWC on libs2v.

Mapping onto the kernels:
  * U-Net ResBlocks (gfpganv1_clean_arch.py:131-149): conv1+lrelu, bilinear resize, the 1x1 skip
    conv writes the block output and conv2+lrelu adds onto it in its epilogue (res after act);
  * SFT condition branches: the first convs of condition_scale[i] and condition_shift[i] read the
    same feature, so they run as ONE conv with both weight sets stacked (2c outputs);
  * modulated convs as in the ENet engine: shared packed weights, input modulation as the
    gather prologue (in_scale), demodulation x sqrt(2) as the per-(n, o) epilogue scale, noise
    (stored buffer or N(0,1)) and bias in the same epilogue;
  * SFT on half the channels (:103-112): one elementwise pass in place on the channel slice.
"""
from __future__ import annotations

import math
import os

import torch

from .. import ops
from ..ops import NHWC, ConvW
from .enet import StyleLayer

LRELU = 0.2
# SFT (gfpganv1_clean_arch.py:98-106: out[:, half:] = out[:, half:] * scale + shift) folded into the StyleConv's
# epilogue (ops.conv2d post=); S2V_GFPGAN_FOLD_SFT=0: a separate elementwise pass
FOLD_SFT = os.environ.get("S2V_GFPGAN_FOLD_SFT", "1") == "1"
# ToRGB and its bilinear x2 skip upsample as one pass (ops.torgb_up2, as ENet's); S2V_GFPGAN_FUSED_TORGB=0:
# resize + small conv with the residual
FUSED_TORGB = os.environ.get("S2V_GFPGAN_FUSED_TORGB", "1") == "1"


class GFPGANEngine:
    def __init__(self, sd, device, num_style_feat=512, sft_half=True, different_w=True, input_is_latent=True):
        if not input_is_latent:
            raise NotImplementedError("GFPGANv1Clean(input_is_latent=False): GFPGANer builds it with True "
                                      "(gfpgan/utils.py:40-50)")
        dev = torch.device(device)
        self.device, self.nsf, self.sft_half, self.different_w = dev, num_style_feat, sft_half, different_w
        w0 = sd["conv_body_first.weight"].float()
        self.first = ConvW(ops.pad_cin(w0, 4), sd["conv_body_first.bias"], dev)
        self.size = None
        nd = sum(1 for k in sd if k.startswith("conv_body_down.") and k.endswith(".conv1.weight"))
        self.levels = nd
        self.log_size = nd + 2

        def resblock(p):
            return (ConvW(sd[p + "conv1.weight"], sd[p + "conv1.bias"], dev, padding=1),
                    ConvW(sd[p + "conv2.weight"], sd[p + "conv2.bias"], dev, padding=1),
                    ConvW(sd[p + "skip.weight"], None, dev))
        self.down = [resblock(f"conv_body_down.{i}.") for i in range(nd)]
        self.up = [resblock(f"conv_body_up.{i}.") for i in range(nd)]
        self.final_conv = ConvW(sd["final_conv.weight"], sd["final_conv.bias"], dev, padding=1)
        wl = sd["final_linear.weight"].float()            # consumes the NCHW flatten (c, h, w)
        c4 = sd["final_conv.weight"].shape[0]
        wl = wl.reshape(wl.shape[0], c4, 4, 4).permute(0, 2, 3, 1).reshape(wl.shape[0], -1)
        self.final_linear = ConvW(wl, sd["final_linear.bias"], dev)
        self.cond = []
        for i in range(nd):
            s, t = f"condition_scale.{i}.", f"condition_shift.{i}."
            first = ConvW(torch.cat([sd[s + "0.weight"], sd[t + "0.weight"]]),
                          torch.cat([sd[s + "0.bias"], sd[t + "0.bias"]]), dev, padding=1)
            self.cond.append((first, ConvW(sd[s + "2.weight"], sd[s + "2.bias"], dev, padding=1),
                              ConvW(sd[t + "2.weight"], sd[t + "2.bias"], dev, padding=1)))
        self.to_rgb_unet = [ConvW(sd[f"toRGB.{i}.weight"], sd[f"toRGB.{i}.bias"], dev) for i in range(nd)]
        d = "stylegan_decoder."
        self.const = sd[d + "constant_input.weight"].float().permute(0, 2, 3, 1).contiguous().to(dev)
        # decoder layers in latent order: style_conv1, to_rgb1, then (conv up, conv, to_rgb) per level
        self.conv1 = StyleLayer(sd, d + "style_conv1.", dev, True, False, False)
        self.rgb1 = StyleLayer(sd, d + "to_rgb1.", dev, False, False, True)
        self.convs = [StyleLayer(sd, f"{d}style_convs.{j}.", dev, True, j % 2 == 0, False) for j in range(2 * nd)]
        self.rgbs = [StyleLayer(sd, f"{d}to_rgbs.{i}.", dev, False, False, True) for i in range(nd)]
        # every decoder layer's style modulation (a Linear on its own 512-d latent, different_w,
        # stylegan2_clean_arch.py:66-99) as ONE segmented GEMV launch (ops.adain_params, the kernel of
        # LNet's ADAIN bank) instead of one small conv per layer: layer L's s is columns
        # [style_off[L], + L.cin) of its output, segment = the layer's latent index
        order = [(self.conv1, 0), (self.rgb1, 1)]
        for lvl in range(nd):
            i = 1 + 2 * lvl
            order += [(self.convs[2 * lvl], i), (self.convs[2 * lvl + 1], i + 1), (self.rgbs[lvl], i + 2)]
        ws, bs, segs, self.style_off, off = [], [], [], {}, 0
        for L, j in order:
            ws.append(L.mod_w)
            bs.append(L.mod_b)
            segs.append(torch.full((L.cin,), j if different_w else 0, dtype=torch.int32))
            self.style_off[id(L)] = off
            off += L.cin
        self.style_w2t = torch.cat(ws, 0).t().contiguous().to(dev)         # [num_style_feat, total]
        self.style_b = torch.cat(bs).contiguous().to(dev)
        self.style_seg = torch.cat(segs).contiguous().to(dev)
        self.style_total = off
        # every demodulated layer's d (style_conv1 + style_convs) from one launch right after the style
        # GEMV (stylegan2_clean_arch.py:81-83 per layer in the reference): layer L's d is columns
        # [demod_r0[L], + L.cout) of the [B, nrows] output
        dl = [self.conv1] + self.convs
        self.demod = ops.DemodRows([(self.style_off[id(L)], L.wsq) for L in dl], dev)
        self.demod_r0 = {id(L): r for L, r in zip(dl, self.demod.r0)}
        self.noise_bufs = [sd[f"{d}noises.noise{i}"].float().reshape(-1).to(dev) for i in range(2 * nd + 1)]
        self._noise_cache = {}
        self.noise_seed = 0x6F9A

    def _stored_noise(self, b):
        """Stored noise buffers [1,1,H,W] broadcast over the batch (randomize_noise=False)."""
        if b not in self._noise_cache:
            self._noise_cache[b] = [t.reshape(1, -1).expand(b, -1).contiguous() for t in self.noise_bufs]
        return self._noise_cache[b]

    def _resblock(self, ctx, x: NHWC, blk, scale):
        c1, c2, sk = blk
        b, dev = x.n, self.device
        oh, ow = int(x.h * scale), int(x.w * scale)
        t = NHWC.empty(b, x.h, x.w, c1.cout, dev)
        ops.conv2d(ctx, x, c1, t, act=ops.ACT_LRELU, alpha=LRELU)
        tr = NHWC.empty(b, oh, ow, c1.cout, dev)
        ops.resize_nhwc(ctx, t, tr, scale_factor=scale)
        xr = NHWC.empty(b, oh, ow, x.c, dev)
        ops.resize_nhwc(ctx, x, xr, scale_factor=scale)
        out = NHWC.empty(b, oh, ow, c2.cout, dev)
        ops.conv2d(ctx, xr, sk, out)
        ops.conv2d(ctx, tr, c2, out, act=ops.ACT_LRELU, alpha=LRELU, res=out, res_after=True)
        return out

    def _style(self, L, sall):
        """Layer L's modulation s [B, cin] (a column range of the bank output ``sall``)."""
        o = self.style_off[id(L)]
        return sall[:, o: o + L.cin]

    def _style_conv(self, ctx, L, x: NHWC, sall, dall, noise, post=None):
        b, dev = x.n, self.device
        s = self._style(L, sall)
        if L.upsample:
            xu = NHWC.empty(b, 2 * x.h, 2 * x.w, x.c, dev)
            ops.resize_nhwc(ctx, x, xu, scale_factor=2)
            x = xu
        r0 = self.demod_r0[id(L)]
        d = dall[:, r0: r0 + L.cout]
        y = NHWC.empty(b, x.h, x.w, L.cout, dev)
        ops.conv2d(ctx, x, L.conv, y, in_scale=s, nc_scale=d, act=ops.ACT_LRELU, alpha=LRELU,
                   pix_add=noise if L.noise_w else None, pix_w=L.noise_w or 0.0, post=post)
        return y

    def forward(self, ctx, x: torch.Tensor, out: torch.Tensor, return_rgb=True, randomize_noise=True, noises=None):
        """x [B,3,S,S] NCHW device tensor -> out [B,3,S,S] (written), list of U-Net RGBs (NCHW)."""
        dev = self.device
        b, _, S, _ = x.shape
        assert S == 2 ** self.log_size, f"GFPGAN engine built for {2 ** self.log_size}x{2 ** self.log_size} inputs"
        x4 = NHWC.empty(b, S, S, 4, dev)
        ops.fill(ctx, x4.t)
        ops.nchw_to_nhwc(ctx, x, x4.slice(0, 3))
        f = NHWC.empty(b, S, S, self.first.cout, dev)
        ops.conv2d(ctx, x4, self.first, f, act=ops.ACT_LRELU, alpha=LRELU)
        skips = []
        for blk in self.down:
            f = self._resblock(ctx, f, blk, 0.5)
            skips.insert(0, f)
        feat = NHWC.empty(b, f.h, f.w, self.final_conv.cout, dev)
        ops.conv2d(ctx, f, self.final_conv, feat, act=ops.ACT_LRELU, alpha=LRELU)
        style = NHWC.empty(b, 1, 1, self.final_linear.cout, dev)
        ops.conv2d(ctx, NHWC(feat.t.view(b, 1, 1, -1)), self.final_linear, style)
        conds, rgbs = [], []
        for i in range(self.levels):
            xin = NHWC.empty(b, feat.h, feat.w, feat.c, dev)
            ops.eltwise(ctx, feat, xin, add=skips[i])
            feat = self._resblock(ctx, xin, self.up[i], 2)
            first, sc2, sh2 = self.cond[i]
            h = NHWC.empty(b, feat.h, feat.w, first.cout, dev)
            ops.conv2d(ctx, feat, first, h, act=ops.ACT_LRELU, alpha=LRELU)
            c = feat.c
            scale = NHWC.empty(b, feat.h, feat.w, sc2.cout, dev)
            ops.conv2d(ctx, h.slice(0, c), sc2, scale)
            shift = NHWC.empty(b, feat.h, feat.w, sh2.cout, dev)
            ops.conv2d(ctx, h.slice(c, c), sh2, shift)
            conds.append((scale, shift))
            if return_rgb:
                r = NHWC.empty(b, feat.h, feat.w, 3, dev)
                ops.conv2d(ctx, feat, self.to_rgb_unet[i], r)
                rn = torch.empty((b, 3, feat.h, feat.w), device=dev)
                ops.nhwc_to_nchw(ctx, r, rn)
                rgbs.append(rn)
        # ---- StyleGAN2 decoder with SFT (gfpganv1_clean_arch.py:89-117)
        nsf = self.nsf

        sall = ops.empty((b, self.style_total), dev)
        ops.adain_params(ctx, style.t.view(b, -1), nsf, self.style_w2t, self.style_b, self.style_seg, sall)
        dall = ops.empty((b, self.demod.nrows), dev)
        ops.modconv_demod_rows(ctx, sall, self.demod, dall, eps=1e-8, post=math.sqrt(2.0))
        nl = 2 * self.levels + 1
        if noises is not None:
            noise = [None if t is None else t.reshape(b, -1).contiguous() for t in noises]
        elif randomize_noise:
            ctr = ctx.noise(id(self)).bump(ctx)            # fresh draws per call, also under graph replay
            noise = []
            for j in range(nl):
                r = 2 ** ((j + 5) // 2)
                t = torch.empty((b, r * r), device=dev)
                ops.gaussian_noise(ctx, t, self.noise_seed, j << 34, ctr=ctr, shift=40)
                noise.append(t)
        else:
            noise = self._stored_noise(b)
        cur = NHWC(self.const.expand(b, -1, -1, -1).contiguous())
        cur = self._style_conv(ctx, self.conv1, cur, sall, dall, noise[0])
        skip = NHWC.empty(b, cur.h, cur.w, 4, dev)             # RGB + a 4th channel the fused ToRGB carries
        ops.fill(ctx, skip.t)
        s = self._style(self.rgb1, sall)
        ops.conv2d(ctx, cur, self.rgb1.conv, skip.slice(0, 3), in_scale=s)
        i = 1
        for lvl in range(self.levels):
            post = None
            if i < 2 * len(conds):
                scale, shift = conds[(i - 1) // 2]
                c = self.convs[2 * lvl].cout
                half = c // 2 if self.sft_half else 0
                post = (scale, shift, half)
            if FOLD_SFT:                                      # the SFT in the StyleConv's epilogue
                cur = self._style_conv(ctx, self.convs[2 * lvl], cur, sall, dall, noise[2 * lvl + 1], post=post)
            else:
                cur = self._style_conv(ctx, self.convs[2 * lvl], cur, sall, dall, noise[2 * lvl + 1])
                if post is not None:
                    part = cur.slice(post[2], cur.c - post[2])
                    ops.eltwise(ctx, part, part, mul=post[0], add=post[1])
            cur = self._style_conv(ctx, self.convs[2 * lvl + 1], cur, sall, dall, noise[2 * lvl + 2])
            R = self.rgbs[lvl]
            rgb = NHWC.empty(b, cur.h, cur.w, 4, dev)
            s = self._style(R, sall)
            if FUSED_TORGB and R.cin % 32 == 0 and (cur.h * cur.w) % 32 == 0:
                ops.torgb_up2(ctx, cur, R.conv, s, skip, rgb)       # ToRGB + bilinear x2 skip (stylegan2_clean_arch.py:157-176)
            else:
                ops.resize_nhwc(ctx, skip, rgb, scale_factor=2)
                ops.conv2d(ctx, cur, R.conv, rgb.slice(0, 3), in_scale=s, res=rgb.slice(0, 3))
            skip = rgb
            i += 2
        ops.nhwc_to_nchw(ctx, skip.slice(0, 3), out)
        return out, rgbs
