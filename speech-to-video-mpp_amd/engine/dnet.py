"""DNet engine (reference models/DNet.py:13-118): MappingNet -> WarpingNet (ADAIN hourglass ->
flow -> fused warp) -> EditingNet.

The hourglass skip concatenations (base_blocks.py:353) are channel slices: each encoder level
writes its output straight into the decoder's [out | skip] buffer.  The dead first branch of
FineADAINResBlock2d (conv1/norm1, base_blocks.py:174 — overwritten on :175) is not computed.
"""
from __future__ import annotations

import torch

from .. import ops
from ..ops import NHWC, ConvW
from .common import AdainBank, make_conv
from .lnet import ROWPACK, ConvNormAct

LRELU = 0.1  # DNet.py:35, :69, :105


class DNetEngine:
    def __init__(self, sd, device):
        dev = torch.device(device)
        self.device = dev
        m = "mapping_net."
        self.map_first = ConvW(sd[m + "first.0.weight"], sd[m + "first.0.bias"], dev)
        self.map_enc = [ConvW(sd[f"{m}encoder{i}.1.weight"], sd[f"{m}encoder{i}.1.bias"], dev, dilation=(1, 3))
                        for i in range(3)]
        self.desc_nc = self.map_first.cout
        self.bank = AdainBank(self.desc_nc)
        h = "warpping_net.hourglass."
        self.input_layer = make_conv(sd, h + "encoder.input_layer.", dev, padding=3)
        if ROWPACK and self.input_layer.cin * self.input_layer.kw <= 64:
            self.input_layer.make_rowpack(dev)         # 7x7 over the RGB source: row-tap packed 7x1 conv
        self.enc = []
        for i in range(5):
            e = f"{h}encoder.encoder{i}."
            c0 = make_conv(sd, e + "conv_0.", dev, stride=2, padding=1)
            c1 = make_conv(sd, e + "conv_1.", dev, padding=1)
            self.enc.append(dict(c0=c0, c1=c1, n0=self._adain(sd, e + "norm_0.", c0.cin),
                                 n1=self._adain(sd, e + "norm_1.", c1.cin)))
        self.dec = []
        for i in (4, 3, 2):
            d = f"{h}decoder.decoder{i}."
            tp = dict(transposed=True, stride=2, padding=1, output_padding=1)
            c0 = make_conv(sd, d + "conv_0.", dev, padding=1)
            c1 = make_conv(sd, d + "conv_1.", dev, **tp).make_polyphase(dev)
            cs = make_conv(sd, d + "conv_s.", dev, **tp).make_polyphase(dev)
            self.dec.append(dict(c0=c0, c1=c1, cs=cs, n0=self._adain(sd, d + "norm_0.", c0.cin),
                                 n1=self._adain(sd, d + "norm_1.", c1.cin), ns=self._adain(sd, d + "norm_s.", cs.cin)))
        f = "warpping_net.flow_out."
        self.flow_ln = (sd[f + "0.weight"].float().reshape(-1).contiguous().to(dev),
                        sd[f + "0.bias"].float().reshape(-1).contiguous().to(dev))
        self.flow_conv = make_conv(sd, f + "2.", dev, padding=3)
        en = "editing_net.encoder."
        self.e_first = ConvNormAct(sd, en + "first.", dev, 7)
        self.e_down = [ConvNormAct(sd, f"{en}down{i}.", dev, 3, pool=True) for i in range(3)]
        de = "editing_net.decoder."
        self.e_dec = []
        for i in (2, 1, 0):
            res = []
            for j in range(2):
                r = f"{de}res{i}.res{j}."
                c2 = make_conv(sd, r + "conv2.", dev, padding=1)
                res.append((c2, self._adain(sd, r + "norm2.", c2.cout)))
            self.e_dec.append(dict(res=res, up=ConvNormAct(sd, f"{de}up{i}.", dev, 3, up=True),
                                   jump=ConvNormAct(sd, f"{de}jump{i}.", dev, 3)))
        self.e_final = make_conv(sd, de + "final.model.0.", dev, padding=3)
        self.bank.build(dev)
        self._pool = {}

    def _adain(self, sd, p, c):
        return self.bank.add_group(sd, [(p, c)])

    def _norm_act(self, ctx, ap, x: NHWC, gid, out: NHWC | None = None, act=ops.ACT_LRELU, res=None):
        """ADAIN ``gid`` (gamma / beta from the bank output ``ap``) + act (+ res)."""
        if out is None:
            out = NHWC.empty(x.n, x.h, x.w, x.c, self.device)
        g, b = self.bank.gamma_beta(gid, ap)
        ops.instnorm(ctx, x, out, g, b, act=act, alpha=LRELU, res=res)
        return out

    def _conv(self, ctx, x: NHWC, cw: ConvW, out: NHWC | None = None, **kw):
        if out is None:
            oh, ow = cw.out_hw(x.h, x.w)
            out = NHWC.empty(x.n, oh, ow, cw.cout, self.device)
        ops.conv2d(ctx, x, cw, out, **kw)
        return out

    def mapping(self, ctx, coeff: torch.Tensor) -> NHWC:
        """MappingNet (DNet.py:48-54): coeff [B,73,L] -> descriptor NHWC [B,1,1,256]."""
        dev = self.device
        b, c, L = coeff.shape
        x = NHWC.empty(b, 1, L, c, dev)
        ops.resize(ctx, coeff, 0, (b, c, 1, L), (coeff.stride(0), coeff.stride(1), 0, coeff.stride(2)),
                   x.t, x.coff, (1, L), ops.nhwc_strides(x))
        out = self._conv(ctx, x, self.map_first)
        for cw in self.map_enc:
            # y = conv(lrelu(out)) + out[:, :, 3:-3]
            out = self._conv(ctx, out, cw, pre_act=ops.ACT_LRELU, pre_alpha=LRELU, res=out, res_offset=(0, 3))
        L2 = out.w
        if L2 not in self._pool:   # AdaptiveAvgPool1d(1) as a 1 x L conv with weight I/L
            self._pool[L2] = ConvW(torch.eye(self.desc_nc)[:, :, None, None].repeat(1, 1, 1, L2) / L2, None, dev)
        return self._conv(ctx, out, self._pool[L2])

    def forward(self, ctx, img: torch.Tensor, coeff: torch.Tensor, stage=None, aux=None):
        dev = self.device
        b, _, H, W = img.shape
        desc = self.mapping(ctx, coeff)
        ap = self.bank.run(ctx, desc)                   # every ADAIN's gamma / beta (descriptor-conditioned)
        # ---- WarpingNet hourglass (base_blocks.py:308-365)
        src = NHWC.empty(b, H, W, 3, dev)
        ops.nchw_to_nhwc(ctx, img, src)
        sizes = [(H >> k, W >> k) for k in range(6)]
        enc_c = [self.input_layer.cout] + [e["c1"].cout for e in self.enc]
        # decoder cat buffers [dec_out | skip]: level k output (k = 3, 2, 1 skips)
        cats = {}
        for k, dd in zip((4, 3, 2), self.dec):
            hh, ww = sizes[k]
            cats[k] = NHWC.empty(b, hh, ww, dd["c1"].cout + enc_c[k], dev)
        x = self._conv(ctx, src, self.input_layer)
        for i, e in enumerate(self.enc):
            t = self._norm_act(ctx, ap, x, e["n0"])
            t = self._conv(ctx, t, e["c0"])
            t = self._norm_act(ctx, ap, t, e["n1"], out=t)
            lvl = i + 1
            dst = cats[lvl].slice(cats[lvl].c - enc_c[lvl], enc_c[lvl]) if lvl in cats else None
            x = self._conv(ctx, t, e["c1"], out=dst)
        cur = x                                          # 256 @ H/32
        for k, d in zip((4, 3, 2), self.dec):
            xs_in = self._norm_act(ctx, ap, cur, d["ns"])
            out = cats[k].slice(0, d["c1"].cout)
            self._conv(ctx, xs_in, d["cs"], out=out)      # x_s = conv_s(actvn(norm_s(x)))
            t = self._norm_act(ctx, ap, cur, d["n0"])
            t = self._conv(ctx, t, d["c0"])
            t = self._norm_act(ctx, ap, t, d["n1"], out=t)
            self._conv(ctx, t, d["c1"], out=out, res=out)  # x_s + dx
            cur = cats[k]
        hg = cur                                         # 256 @ H/4
        t = NHWC.empty(b, hg.h, hg.w, hg.c, dev)
        ops.layernorm2d(ctx, hg, *self.flow_ln, t, act=ops.ACT_LRELU, alpha=LRELU)
        flow = self._conv(ctx, t, self.flow_conv)        # [B, H/4, W/4, 2]
        x6 = NHWC.empty(b, H, W, 6, dev)
        ops.flow_warp_cat(ctx, flow, img, x6)            # [img | warp(img)] (DNet.py:89, :114-115)
        result = {"flow_field": torch.empty((b, 2, flow.h, flow.w), device=dev),
                  "warp_image": torch.empty((b, 3, H, W), device=dev)}
        ops.nhwc_to_nchw(ctx, flow, result["flow_field"])
        ops.nhwc_to_nchw(ctx, x6.slice(3, 3), result["warp_image"])
        if aux is not None:
            aux["descriptor"] = desc.t.view(b, -1)
        if stage == "warp":
            return result
        # ---- EditingNet (DNet.py:114-118, base_blocks.py:255-305)
        f0 = self.e_first(ctx, x6)
        skips = [f0]
        x = f0
        for i, dn in enumerate(self.e_down):
            x = dn(ctx, x)
            if i < 2:
                skips.append(x)
        out = x
        for lv in self.e_dec:
            for c2, gid in lv["res"]:
                t = self._conv(ctx, out, c2)
                self._norm_act(ctx, ap, t, gid, out=out, act=ops.ACT_NONE, res=out)   # norm2(conv2(x)) + x
            up = lv["up"](ctx, out)
            lv["jump"](ctx, skips.pop(), out=up, res=up)
            out = up
        fake = NHWC.empty(b, H, W, 3, dev)
        ops.conv2d(ctx, out, self.e_final, fake, act=ops.ACT_TANH)
        result["fake_image"] = torch.empty((b, 3, H, W), device=dev)
        ops.nhwc_to_nchw(ctx, fake, result["fake_image"])
        return result
