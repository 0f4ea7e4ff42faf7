"""GPEN FullGenerator engine (third_part/GPEN/face_model/gpen_model.py:386-630), NHWC on libs2v.

Equalized-learning-rate scales, FusedLeakyReLU's sqrt(2) gain and the style-MLP lr_mul are folded
into the packed weights / biases once (lrelu is positively homogeneous, so
sqrt(2) * lrelu(v + b) == lrelu(sqrt(2) v + sqrt(2) b)).  Per layer:
  * encoder ConvLayer(downsample): NHWC FIR blur (s2v_fir2d, pad 2) -> stride-2 conv with
    bias + lrelu in the epilogue (gpen_model.py:515-562);
  * StyledConv (isconcat=True): the modulated conv writes channels [0, C) of a 2C buffer with
    demod * sqrt(2), bias and lrelu fused; NoiseInjection's concat half lrelu(sqrt(2) (w * e + b))
    of the encoder feature e is one elementwise pass into channels [C, 2C) (:292-363);
  * upsampling StyledConv: transposed stride-2 conv (modulation as prologue, demod as epilogue),
    then the FIR blur with bias + lrelu fused, writing straight into the concat slice (:262-276);
  * ToRGB: FIR x2 upsample of the skip into the output buffer, then the 1x1 modulated conv adds
    onto it in its epilogue (:374-384);
  * all modulations consume the same latent: one GEMM for every layer (segments padded to 4);
  * PixelNorm (:18-23) is folded into the first style-MLP GEMM as a per-sample epilogue scale
    rsqrt(mean(x^2) + 1e-8), computed by the demodulation kernel with a 1/512 weight table.
"""
from __future__ import annotations

import math
import os

import torch

from .. import ops
from ..ops import NHWC, ConvW

LRELU = 0.2
SQ2 = math.sqrt(2.0)
# NoiseInjection's concat half (gpen_model.py:292-302): S2V_GPEN_FOLD_NOISE=1 writes it from the StyledConv's
# epilogue as a second output (ops.conv2d dup=) on the non-upsampling layers.  Off by default: measured 0.4 %
# slower on the enhance workload (the epilogue's extra dependent loads cost the conv more than the separate
# pass costs, MI355X A/B r06)
FOLD_NOISE = os.environ.get("S2V_GPEN_FOLD_NOISE", "0") == "1"


class _StyledLayer:
    def __init__(self, sd, p, dev, upsample, is_rgb):
        w = sd[p + "conv.weight"].float()[0]                  # [O, I, k, k]
        o, i, k, _ = w.shape
        w = w / math.sqrt(i * k * k)                          # ModulatedConv2d.scale (:231-233)
        self.cin, self.cout, self.k, self.upsample, self.is_rgb = i, o, k, upsample, is_rgb
        if upsample:
            self.conv = ConvW(w.transpose(0, 1), None, dev, transposed=True, stride=2, padding=0).make_polyphase(dev)
            self.blur = sd[p + "conv.blur.kernel"].float().contiguous().to(dev)
        else:
            self.conv = ConvW(w, None, dev, padding=k // 2)
        self.wsq = w.pow(2).sum((2, 3)).contiguous().to(dev)
        wm = sd[p + "conv.modulation.weight"].float()
        self.mod_w = wm / math.sqrt(wm.shape[1])             # EqualLinear scale, lr_mul 1
        self.mod_b = sd[p + "conv.modulation.bias"].float()
        if is_rgb:
            self.bias = sd[p + "bias"].float().reshape(-1).contiguous().to(dev)
            self.up_k = sd[p + "upsample.kernel"].float().contiguous().to(dev) if p + "upsample.kernel" in sd else None
        else:
            b = sd[p + "activate.bias"].float() * SQ2
            self.bias_a = b[:o].contiguous().to(dev)
            self.bias_n = b[o:].contiguous().to(dev)
            self.noise_w = float(sd[p + "noise.weight"].float().reshape(-1)[0])
        self.mod_off = 0


class GPENEngine:
    def __init__(self, sd, device, n_mlp=8, lr_mlp=0.01):
        dev = torch.device(device)
        self.device = dev
        self.log_size = sum(1 for k in sd if k.startswith("ecd") and k.endswith(".bias")) + 1
        # encoder (FullGenerator.ecd*, gpen_model.py:597-604)
        w = sd["ecd0.0.0.weight"].float()
        self.ecd0 = ConvW(ops.pad_cin(w / math.sqrt(w[0].numel()) * SQ2, 4), sd["ecd0.0.1.bias"].float() * SQ2, dev)
        self.ecd = []
        for i in range(1, self.log_size - 1):
            p = f"ecd{i}.0."
            w = sd[p + "1.weight"].float()
            self.ecd.append((sd[p + "0.kernel"].float().contiguous().to(dev),
                             ConvW(w / math.sqrt(w[0].numel()) * SQ2, sd[p + "2.bias"].float() * SQ2, dev,
                                   stride=2, padding=0)))
        wl = sd["final_linear.0.weight"].float()
        c4 = self.ecd[-1][1].cout
        wl = wl.reshape(wl.shape[0], c4, 4, 4).permute(0, 2, 3, 1).reshape(wl.shape[0], -1)
        self.final_linear = ConvW(wl / math.sqrt(wl.shape[1]) * SQ2, sd["final_linear.0.bias"].float() * SQ2, dev)
        # style MLP (Generator.style, :404-412): PixelNorm + n_mlp EqualLinear(lr_mul) + fused lrelu
        g = "generator."
        self.mlp = []
        for i in range(1, n_mlp + 1):
            w = sd[f"{g}style.{i}.weight"].float()
            self.mlp.append(ConvW(w * (lr_mlp / math.sqrt(w.shape[1])) * SQ2,
                                  sd[f"{g}style.{i}.bias"].float() * lr_mlp * SQ2, dev))
        sdim = self.mlp[0].cin
        self.pn_table = torch.full((self.mlp[0].cout, sdim), 1.0 / sdim, device=dev)
        self.const = sd[g + "input.input"].float().permute(0, 2, 3, 1).contiguous().to(dev)
        self.conv1 = _StyledLayer(sd, g + "conv1.", dev, False, False)
        self.rgb1 = _StyledLayer(sd, g + "to_rgb1.", dev, False, True)
        nlev = self.log_size - 2
        self.convs = [_StyledLayer(sd, f"{g}convs.{j}.", dev, j % 2 == 0, False) for j in range(2 * nlev)]
        self.rgbs = [_StyledLayer(sd, f"{g}to_rgbs.{i}.", dev, False, True) for i in range(nlev)]
        # one modulation GEMM for every layer (all consume the same latent, :470-477)
        ws, bs, off = [], [], 0
        for L in [self.conv1, self.rgb1] + self.convs + self.rgbs:
            pad = (-L.cin) % 4
            L.mod_off = off
            ws += [L.mod_w, torch.zeros(pad, L.mod_w.shape[1])]
            bs += [L.mod_b, torch.zeros(pad)]
            off += L.cin + pad
        self.mod = ConvW(torch.cat(ws), torch.cat(bs), dev)
        # every StyledConv's demodulation from one launch after the modulation GEMM (gpen_model.py:225-247
        # per layer in the reference): layer L's d is columns [demod_r0[L], + L.cout) of the output
        dl = [self.conv1] + self.convs
        self.demod = ops.DemodRows([(L.mod_off, L.wsq) for L in dl], dev)
        for L, r in zip(dl, self.demod.r0):
            L.demod_r0 = r

    def _styled(self, ctx, L, x: NHWC, svec, dall, out: NHWC, noise: NHWC):
        """StyledConv with isconcat: out [.., 2C] <- (lrelu(sqrt2 (demod conv + b)), lrelu(sqrt2 (w e + b)))."""
        b, dev = x.n, self.device
        s = svec[:, L.mod_off: L.mod_off + L.cin]
        d = dall[:, L.demod_r0: L.demod_r0 + L.cout]
        C = L.cout
        if L.upsample:
            oh, ow = L.conv.out_hw(x.h, x.w)
            t = NHWC.empty(b, oh, ow, C, dev)
            ops.conv2d(ctx, x, L.conv, t, in_scale=s, nc_scale=d)
            ops.fir2d(ctx, t, L.blur, out.slice(0, C), pad0=(1, 1), bias=L.bias_a, act=ops.ACT_LRELU, alpha=LRELU)
        elif FOLD_NOISE:
            # the concat half in the same epilogue: out[.., C + n] = lrelu(sqrt2 (w e + b)) of the encoder feature e
            ops.conv2d(ctx, x, L.conv, out.slice(0, C), in_scale=s, nc_scale=d, shift=L.bias_a,
                       act=ops.ACT_LRELU, alpha=LRELU, dup=(noise, L.bias_n, SQ2 * L.noise_w, C))
            return out
        else:
            ops.conv2d(ctx, x, L.conv, out.slice(0, C), in_scale=s, nc_scale=d, shift=L.bias_a,
                       act=ops.ACT_LRELU, alpha=LRELU)
        ops.eltwise(ctx, noise, out.slice(C, C), a=SQ2 * L.noise_w, bias=L.bias_n, act=ops.ACT_LRELU, alpha=LRELU)
        return out

    def forward(self, ctx, x: torch.Tensor, out: torch.Tensor, input_is_latent=False, latent_out=None):
        """x [B,3,S,S] NCHW device tensor in [-1,1] -> out [B,3,S,S] (written)."""
        dev = self.device
        b, _, S, _ = x.shape
        assert S == 2 ** self.log_size, f"GPEN engine built for {2 ** self.log_size}x{2 ** self.log_size} inputs"
        x4 = NHWC.empty(b, S, S, 4, dev)
        ops.fill(ctx, x4.t)
        ops.nchw_to_nhwc(ctx, x, x4.slice(0, 3))
        e = NHWC.empty(b, S, S, self.ecd0.cout, dev)
        ops.conv2d(ctx, x4, self.ecd0, e, act=ops.ACT_LRELU, alpha=LRELU)
        feats = [e]
        for kern, cw in self.ecd:
            bl = NHWC.empty(b, e.h + 1, e.w + 1, e.c, dev)            # Blur pad (2, 2): H + 4 - 4 + 1
            ops.fir2d(ctx, e, kern, bl, pad0=(2, 2))
            oh, ow = cw.out_hw(bl.h, bl.w)
            e = NHWC.empty(b, oh, ow, cw.cout, dev)
            ops.conv2d(ctx, bl, cw, e, act=ops.ACT_LRELU, alpha=LRELU)
            feats.append(e)
        code = NHWC.empty(b, 1, 1, self.final_linear.cout, dev)
        ops.conv2d(ctx, NHWC(e.t.view(b, 1, 1, -1)), self.final_linear, code, act=ops.ACT_LRELU, alpha=LRELU)
        lat = code
        if not input_is_latent:
            r = torch.empty((b, self.mlp[0].cout), device=dev)
            ops.modconv_demod(ctx, code.t.view(b, -1), self.pn_table, r, eps=1e-8, post=1.0)   # PixelNorm
            for j, cw in enumerate(self.mlp):
                nxt = NHWC.empty(b, 1, 1, cw.cout, dev)
                ops.conv2d(ctx, lat, cw, nxt, act=ops.ACT_LRELU, alpha=LRELU, nc_scale=r if j == 0 else None)
                lat = nxt
        if latent_out is not None:
            latent_out.copy_(lat.t.view(b, -1))
        svec = NHWC.empty(b, 1, 1, self.mod.cout, dev)
        ops.conv2d(ctx, lat, self.mod, svec)
        sv = svec.t.view(b, -1)
        dall = ops.empty((b, self.demod.nrows), dev)
        ops.modconv_demod_rows(ctx, sv, self.demod, dall, eps=1e-8, post=SQ2)
        noise = [f for f in feats[::-1] for _ in range(2)][1:]      # FullGenerator.forward (:619-621)
        cur_in = NHWC(self.const.expand(b, -1, -1, -1).contiguous())
        cat = NHWC.empty(b, 4, 4, 2 * self.conv1.cout, dev)
        self._styled(ctx, self.conv1, cur_in, sv, dall, cat, noise[0])
        skip = NHWC.empty(b, 4, 4, 3, dev)
        s = sv[:, self.rgb1.mod_off: self.rgb1.mod_off + self.rgb1.cin]
        ops.conv2d(ctx, cat, self.rgb1.conv, skip, in_scale=s, shift=self.rgb1.bias)
        for lvl in range(self.log_size - 2):
            L1, L2, R = self.convs[2 * lvl], self.convs[2 * lvl + 1], self.rgbs[lvl]
            h = 2 * cat.h
            a = NHWC.empty(b, h, h, 2 * L1.cout, dev)
            self._styled(ctx, L1, cat, sv, dall, a, noise[2 * lvl + 1])
            cat = NHWC.empty(b, h, h, 2 * L2.cout, dev)
            self._styled(ctx, L2, a, sv, dall, cat, noise[2 * lvl + 2])
            rgb = NHWC.empty(b, h, h, 3, dev)
            ops.fir2d(ctx, skip, R.up_k, rgb, up=2, pad0=(2, 2))     # Upsample pad (2, 1)
            s = sv[:, R.mod_off: R.mod_off + R.cin]
            ops.conv2d(ctx, cat, R.conv, rgb, in_scale=s, shift=R.bias, res=rgb)
            skip = rgb
        ops.nhwc_to_nchw(ctx, skip, out)
        return out
