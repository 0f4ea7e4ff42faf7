"""LNet engine: the audio-conditioned lip-sync U-Net (reference models/LNet.py:80-139) on libs2v.

Data layout: NHWC fp32 in HBM.  The reference's torch.cat / split / narrow calls are channel
slices of one buffer (e.g. the 1024-channel [x_maskGT | x_ref] feature at 12x12 is written in
place by the two encoder streams, FFC x_l / x_g are channel ranges of the block tensor).
"""
from __future__ import annotations

import os

import torch

from .. import ops
from ..ops import NHWC, ConvW
from .common import AdainBank, bn_tuple, conv_weight, make_conv

LRELU = 0.1        # LNet.py:91
LRELU_FFC = 0.01   # FineADAINLama built with nn.LeakyReLU() default (base_blocks.py:369 via :393/:419)
# FFC products on concurrent side streams (S2V_LNET_BRANCHES=0 serialises them on one stream)
BRANCHES = os.environ.get("S2V_LNET_BRANCHES", "1") == "1"
# S2V_LNET_GROUP=1: the FFC's three products that read the block input (conv_to_l, l2g, the spectral
# branch's st1) as ONE grouped launch (ops.conv_group / s2v_conv2d_group) followed by the spectral chain
# on the same stream, instead of the three side-stream branches.  Measured on MI355X (r04, 3 interleaved
# pairs): LNet B=16 10.78 ms grouped vs 10.48 ms branched, lipsync 24.31 vs 24.30 ms — the grouped
# launch serialises the spectral chain behind the two big convs, which the branches overlap — so the
# branches stay the default (the up2 polyphase classes use the grouped launch, ops.conv2d).
GROUP = os.environ.get("S2V_LNET_GROUP", "0") == "1"
# FFC 3x3 reflect convs over a pre-padded input (S2V_LNET_PREPAD=0: reflect addressing in the gather)
PREPAD = os.environ.get("S2V_LNET_PREPAD", "1") == "1"
# with PREPAD: the InstanceNorm that ends an FFC writes the next FFC's reflect-padded input itself
FUSED_PAD = os.environ.get("S2V_LNET_FUSED_PAD", "1") == "1"
# nearest-x2 UpBlock convs as four parity-class 2x2 convs of the un-upsampled input
# (ConvW.make_up2_polyphase; S2V_UP2_POLY=0: the upsampling gather of the direct 3x3 conv)
UP2_POLY = os.environ.get("S2V_UP2_POLY", "1") == "1"
# 7x7 convs over <= 8 channels as row-tap packed 7x1 convs (ConvW.make_rowpack + ops.row_pack;
# S2V_ROWPACK=0: the per-element gather of the direct conv)
ROWPACK = os.environ.get("S2V_ROWPACK", "1") == "1"
# split-K factor forced on the FourierUnit chain's 1x1 convs (st1, fu, st2); 0 = the planner's choice.  1 (no
# split-K, no reduce launch on the branch): LNet B=16 11.97 -> 11.69 ms on MI355X (r03), lipsync unchanged
SPEC_SPLITS = int(os.environ.get("S2V_LNET_SPEC_SPLITS", "1"))
# encoder branches: calling stream first, then the two side streams (m = masked face, r = reference
# face, a = audio encoder + ADAIN heads)
ENC_ORDER = os.environ.get("S2V_LNET_ENC_ORDER", "mra")
# the FFC's spectral branch and norm as three fused kernels (ops.ffc_spec_fwd / ffc_spec_inv / ffc_norm,
# csrc/ffc.hip) instead of st1 -> rfft2 -> fu -> irfft2 -> st2 -> instnorm (split-precision arithmetic only;
# S2V_LNET_FUSED=0: the separate launches).  S2V_LNET_FUSED_LEVELS: the decoder levels (h) that take it; on
# MI355X (r05, tools/ffc_micro.py, B = 16) the fused kernels win at 24^2 only: each block streams its whole
# image (the channel slices of an image all read the same A rows), which at 12^2 / 48^2 costs more than
# the launches it saves
FUSED = os.environ.get("S2V_LNET_FUSED", "1") == "1"
FUSED_LEVELS = tuple(int(v) for v in os.environ.get("S2V_LNET_FUSED_LEVELS", "24").split(",") if v)
# S2V_LNET_PAIR=1: conv_to_l and l2g (both read the reflect-padded block input) as ONE grouped launch
# (ops.conv_group) on the calling stream, the spectral chain on a single side stream
PAIR = os.environ.get("S2V_LNET_PAIR", "1") == "1"
# with PAIR: the grouped conv launch on the side stream and the spectral chain on the calling stream
PAIR_SIDE = os.environ.get("S2V_LNET_PAIR_SIDE", "0") == "1"
# split-K forced on the FFC's conv_to_l / l2g at the 12^2 level (0 = the planner's choice)
C2L_SPLITS = int(os.environ.get("S2V_LNET_C2L_SPLITS", "0"))
L2G_SPLITS = int(os.environ.get("S2V_LNET_L2G_SPLITS", "0"))

AUDIO_CFG = [  # LNet.py:102-120: (stride, padding, residual)
    (1, 1, False), (1, 1, True), (1, 1, True), ((3, 1), 1, False), (1, 1, True), (1, 1, True),
    (3, 1, False), (1, 1, True), (1, 1, True), ((3, 2), 1, False), (1, 1, True), (1, 0, False), (1, 0, False)]


class ConvNormAct:
    """conv -> LayerNorm2d -> LeakyReLU (-> avgpool2) (FirstBlock2d/DownBlock2d/UpBlock2d/Jump)."""

    def __init__(self, sd, p, device, k, pool=False, up=False):
        self.conv = make_conv(sd, p + "model.0.", device, padding=k // 2,
                              in_mode=ops.IN_NEAREST_UP2 if up else ops.IN_DIRECT)
        if up and UP2_POLY and k == 3 and self.conv.cin % 32 == 0:
            self.conv.make_up2_polyphase(device)      # 4 parity-class 2x2 convs of the un-upsampled input
        elif not up and ROWPACK and k >= 5 and self.conv.cin * k <= 64:
            self.conv.make_rowpack(device)            # 7x7 over 3 / 6 channels: row-tap packed kh x 1 conv
        self.ln_w = sd[p + "model.1.weight"].float().reshape(-1).contiguous().to(device)
        self.ln_b = sd[p + "model.1.bias"].float().reshape(-1).contiguous().to(device)
        self.pool = pool
        self.device = device

    def out_shape(self, x: NHWC):
        oh, ow = self.conv.out_hw(x.h, x.w)
        if self.pool:
            oh, ow = oh // 2, ow // 2
        return x.n, oh, ow, self.conv.cout

    def __call__(self, ctx, x: NHWC, out: NHWC | None = None, res: NHWC | None = None) -> NHWC:
        oh, ow = self.conv.out_hw(x.h, x.w)
        tmp = NHWC.empty(x.n, oh, ow, self.conv.cout, self.device)
        ops.conv2d(ctx, x, self.conv, tmp)
        if out is None:
            out = NHWC.empty(*self.out_shape(x), self.device)
        ops.layernorm2d(ctx, tmp, self.ln_w, self.ln_b, out, act=ops.ACT_LRELU, alpha=LRELU, pool=self.pool, res=res)
        return out


class Transformer:
    """models/transformer.py:89-112 (DualPreNorm cross attention, q,k <- x, v <- y)."""

    def __init__(self, sd, p, device, depth=2, heads=4, dim_head=64):
        self.layers = []
        self.heads, self.dim_head = heads, dim_head
        t = lambda k: sd[k].float().contiguous().to(device)  # noqa: E731
        for i in range(depth):
            a, f = f"{p}layers.{i}.0.", f"{p}layers.{i}.1."
            self.layers.append(dict(
                nx=(t(a + "normx.weight"), t(a + "normx.bias")), ny=(t(a + "normy.weight"), t(a + "normy.bias")),
                qk=ConvW(torch.cat([sd[a + "fn.to_q.weight"], sd[a + "fn.to_k.weight"]], 0), None, device),
                v=ConvW(sd[a + "fn.to_v.weight"], None, device),
                out=ConvW(sd[a + "fn.to_out.0.weight"], sd[a + "fn.to_out.0.bias"], device),
                nf=(t(f + "norm.weight"), t(f + "norm.bias")),
                ff1=ConvW(sd[f + "fn.net.0.weight"], sd[f + "fn.net.0.bias"], device),
                ff2=ConvW(sd[f + "fn.net.3.weight"], sd[f + "fn.net.3.bias"], device)))
        self.inner = heads * dim_head
        self.device = device

    def __call__(self, ctx, x: NHWC, y: NHWC, out: NHWC):
        """x: dense NHWC [B,h,w,C] scratch (used in place as the residual stream), y: NHWC view
        (tokens = pixels, row stride y.cs); result written to ``out`` (a channel slice)."""
        b, h, w, c = x.n, x.h, x.w, x.c
        assert x.cs == c and x.coff == 0
        T = h * w
        rows = b * T
        dev = self.device
        xt = x.t.view(rows, c)
        yt = y.t.view(rows, y.cs)[:, y.coff: y.coff + c]
        xn = torch.empty_like(xt)
        yn = torch.empty_like(xt)
        qk = torch.empty((rows, 2 * self.inner), device=dev)
        v = torch.empty((rows, self.inner), device=dev)
        o = torch.empty((rows, self.inner), device=dev)
        hdn = torch.empty((rows, self.layers[0]["ff1"].cout), device=dev)
        as4 = lambda t: NHWC(t.view(rows, 1, 1, t.shape[1]))  # noqa: E731
        for li, L in enumerate(self.layers):
            ops.row_layernorm(ctx, xt, *L["nx"], xn)
            ops.row_layernorm(ctx, yt, *L["ny"], yn)
            ops.conv2d(ctx, as4(xn), L["qk"], as4(qk))
            ops.conv2d(ctx, as4(yn), L["v"], as4(v))
            ops.attention(ctx, qk[:, : self.inner], qk[:, self.inner:], v, o, batch=b, heads=self.heads, tokens=T,
                          dim_head=self.dim_head)
            ops.conv2d(ctx, as4(o), L["out"], as4(xt), res=as4(xt))
            ops.row_layernorm(ctx, xt, *L["nf"], xn)
            ops.conv2d(ctx, as4(xn), L["ff1"], as4(hdn), act=ops.ACT_GELU_TANH)
            last = li == len(self.layers) - 1
            dst = NHWC(out.t.view(rows, 1, 1, out.cs), out.coff, c) if last else as4(xt)
            ops.conv2d(ctx, as4(hdn), L["ff2"], dst, res=as4(xt))
        return out


class FFCLama:
    """FineADAINLama (base_blocks.py:368-386) = FFC (ffc.py:176-233, ratio 0.75, reflect 3x3,
    spectral g2g without LFU) + ADAIN(bn_l | bn_g) + LeakyReLU(0.01)."""

    def __init__(self, sd, p, device, c, hw, bank: AdainBank):
        f = p + "ffc."
        self.c = c
        self.cg = int(c * 0.75)
        self.cl = c - self.cg
        self.cc = self.cg // 2
        # reflect-padded 3x3 convs run as valid convs over one reflect-padded copy of the block input
        # (PREPAD): no per-tap reflection in the gather, so they take the buffer-load A path
        rp = dict(padding=0) if PREPAD else dict(padding=1, pad_mode=ops.PAD_REFLECT)
        w_l2l, w_g2l = sd[f + "convl2l.weight"].float(), sd[f + "convg2l.weight"].float()
        self.conv_to_l = ConvW(torch.cat([w_l2l, w_g2l], 1), None, device, **rp)   # l2l(x_l) + g2l(x_g)
        self.conv_l2g = ConvW(sd[f + "convl2g.weight"], None, device, **rp)
        st = f + "convg2g."
        self.st1 = ConvW(sd[st + "conv1.0.weight"], None, device, bn=bn_tuple(sd, st + "conv1.1."))
        # FourierUnit 1x1 conv on [re, im]-interleaved channels (ffc.py:100-118) -> reorder to
        # (part, channel) so the spectrum is a plain [B, F, 2C] tensor.
        cc = self.cc
        perm = torch.tensor([2 * (i % cc) + i // cc for i in range(2 * cc)])
        wfu = sd[st + "fu.conv_layer.weight"].float()[perm][:, perm]
        bn = tuple(t.float()[perm] for t in bn_tuple(sd, st + "fu.bn."))
        self.fu = ConvW(wfu, None, device, bn=bn)
        self.st2 = ConvW(sd[st + "conv2.weight"], None, device)
        self.h, self.w = hw
        self.fft = ops.fft_tables(self.h, self.w, device)
        self.F = self.h * (self.w // 2 + 1)
        self.gid = bank.add_group(sd, [(p + "bn_l.", self.cl), (p + "bn_g.", self.cg)])
        self.device = device

    def fused(self) -> bool:
        return FUSED and not GROUP and self.h in FUSED_LEVELS and ops.ffc_fused_ok()

    @staticmethod
    def _run_products(ctx, branches, c2l, l2g, spectral, grouped):
        """conv_to_l, l2g and the spectral chain: concurrent branches (``branches``), or serial; with
        ``grouped`` (PAIR) the two convs as one grouped launch on the calling stream beside the spectral
        chain on one side stream."""
        if grouped:
            def pair(c):
                with ops.conv_group(c):
                    c2l(c)
                    l2g(c)
            if branches is None:
                pair(ctx)
                spectral(ctx)
            elif PAIR_SIDE:
                branches.run(ctx, spectral, pair)
            else:
                branches.run(ctx, pair, spectral)
        elif branches is None:
            c2l(ctx)
            l2g(ctx)
            spectral(ctx)
        else:
            branches.run(ctx, c2l, l2g, spectral)

    def pre_norm(self, ctx, x: NHWC, y: NHWC, branches=None, xpad: NHWC | None = None):
        """y <- [l2l(x_l)+g2l(x_g) | l2g(x_l) + spectral(x_g)] (before ADAIN).

        The three independent products run as concurrent branches when ``branches`` (two
        (stream, Ctx) pairs, see Branches) is given: conv_to_l on the calling stream, l2g on the
        first side stream, the spectral chain st1 -> rfft2 -> fu -> irfft2 on the second; st2 joins
        them (it accumulates onto l2g's output).  At 12x12 each product fills only a fraction of
        the 256 CUs, so running them side by side is what fills the chip.

        Fused (``self.fused()``): the spectral branch is ops.ffc_spec_fwd + ops.ffc_spec_inv (two launches,
        u = irfft(fu(rfft(t1))) + t1) and st2 moves into ``norm`` (ops.ffc_norm adds u conv2 to l2g's output
        per channel slice before the statistics); returns u, which ``norm`` takes."""
        b = x.n
        cl, cg, cc, dev = self.cl, self.cg, self.cc, self.device
        yg = y.slice(cl, cg)
        if self.fused():
            return self._pre_norm_fused(ctx, x, y, branches, xpad)
        t1 = NHWC.empty(b, self.h, self.w, cc, dev)
        spec = torch.empty((b, self.F, 2 * cc), device=dev)
        spec2 = NHWC.empty(b, self.F, 1, 2 * cc, dev)
        u = NHWC.empty(b, self.h, self.w, cc, dev)

        xr = x
        if PREPAD and xpad is not None:
            xr = xpad                                  # written by the previous InstanceNorm (norm(pad_out=))
        elif PREPAD:
            xr = NHWC.empty(b, self.h + 2, self.w + 2, x.c, dev)
            ops.pad_reflect(ctx, x, xr, (1, 1, 1, 1))

        small = self.h <= 12
        fs_l2g = L2G_SPLITS if small else 0
        fs_c2l = C2L_SPLITS if small else 0

        def l2g(c):
            ops.conv2d(c, xr.slice(0, cl), self.conv_l2g, yg, force_splits=fs_l2g)

        def spectral(c):
            ops.conv2d(c, x.slice(cl, cg), self.st1, t1, act=ops.ACT_RELU, force_splits=SPEC_SPLITS)
            ops.rfft2(c, t1, self.fft, spec)                             # rfftn ortho (ffc.py:99-104)
            ops.conv2d(c, NHWC(spec.view(b, self.F, 1, 2 * cc)), self.fu, spec2, act=ops.ACT_RELU,
                       force_splits=SPEC_SPLITS)
            ops.irfft2(c, spec2.t.view(b, self.F, 2 * cc), self.fft, u, res=t1)   # irfftn + x (ffc.py:120-126, :158)

        if GROUP and not fs_c2l and not fs_l2g:
            with ops.conv_group(ctx):
                ops.conv2d(ctx, xr, self.conv_to_l, y.slice(0, cl))
                l2g(ctx)
                ops.conv2d(ctx, x.slice(cl, cg), self.st1, t1, act=ops.ACT_RELU)
            ops.rfft2(ctx, t1, self.fft, spec)
            ops.conv2d(ctx, NHWC(spec.view(b, self.F, 1, 2 * cc)), self.fu, spec2, act=ops.ACT_RELU,
                       force_splits=SPEC_SPLITS)
            ops.irfft2(ctx, spec2.t.view(b, self.F, 2 * cc), self.fft, u, res=t1)
        else:
            self._run_products(ctx, branches,
                               lambda c: ops.conv2d(c, xr, self.conv_to_l, y.slice(0, cl), force_splits=fs_c2l), l2g,
                               spectral, PAIR and not fs_c2l and not fs_l2g)
        ops.conv2d(ctx, u, self.st2, yg, res=yg, force_splits=SPEC_SPLITS)
        return None

    def _pre_norm_fused(self, ctx, x: NHWC, y: NHWC, branches, xpad):
        b = x.n
        cl, cg, cc, dev = self.cl, self.cg, self.cc, self.device
        yg = y.slice(cl, cg)
        t1 = NHWC.empty(b, self.h, self.w, cc, dev)
        spec = torch.empty((b, self.F, 2 * cc), device=dev)
        u = NHWC.empty(b, self.h, self.w, cc, dev)
        xr = x
        if PREPAD and xpad is not None:
            xr = xpad
        elif PREPAD:
            xr = NHWC.empty(b, self.h + 2, self.w + 2, x.c, dev)
            ops.pad_reflect(ctx, x, xr, (1, 1, 1, 1))
        small = self.h <= 12
        fs_l2g = L2G_SPLITS if small else 0
        fs_c2l = C2L_SPLITS if small else 0

        def c2l(c):
            ops.conv2d(c, xr, self.conv_to_l, y.slice(0, cl), force_splits=fs_c2l)

        def l2g(c):
            ops.conv2d(c, xr.slice(0, cl), self.conv_l2g, yg, force_splits=fs_l2g)

        def spectral(c):
            ops.ffc_spec_fwd(c, x.slice(cl, cg), self.st1, self.fft, t1, spec)   # st1 + rfftn (ffc.py:98-104, :158)
            ops.ffc_spec_inv(c, spec, self.fu, self.fft, t1, u)                  # fu + irfftn + x (ffc.py:106-126)

        self._run_products(ctx, branches, c2l, l2g, spectral, PAIR and not fs_c2l and not fs_l2g)
        return u

    def norm(self, ctx, bank: AdainBank, params, y: NHWC, out: NHWC, res: NHWC | None = None,
             pad_out: NHWC | None = None, u: NHWC | None = None):
        """ADAIN(bn_l | bn_g) + LeakyReLU (+ residual); with ``u`` (the fused pre_norm's FourierUnit output)
        the spectral branch's st2 conv is added to y's global channels first (ops.ffc_norm)."""
        g, bt = bank.gamma_beta(self.gid, params)
        if u is not None:
            ops.ffc_norm(ctx, y, u, self.st2, out, g, bt, act=ops.ACT_LRELU, alpha=LRELU_FFC, res=res, pad_out=pad_out)
        else:
            ops.instnorm(ctx, y, out, g, bt, act=ops.ACT_LRELU, alpha=LRELU_FFC, res=res, pad_out=pad_out)


class Branches:
    """Fork / join of independent work on side HIP streams (captured into the same graph when the
    caller is capturing: the side streams fork from and join back into the calling stream).  The
    streams and their Ctx objects belong to the calling lane (``ops.Ctx.streams``), so split-K
    workspaces never alias across concurrent launches or across lanes."""

    def __init__(self, device, side):
        self.device = torch.device(device)
        self.side = side

    def run(self, ctx, main, *others):
        cur = torch.cuda.current_stream(self.device)
        for st, _ in self.side[: len(others)]:
            st.wait_stream(cur)
        keep = ctx.keep                          # side-branch tensors: calling-stream memory (ops.side_stream)
        for (st, c), fn in zip(self.side, others):
            with ops.side_stream(st, keep):
                fn(c)
        main(ctx)
        for st, _ in self.side[: len(others)]:
            cur.wait_stream(st)


class LNetEngine:
    def __init__(self, sd, device, prefix=""):
        p = prefix
        dev = torch.device(device)
        self.device = dev
        e = p + "encoder."
        self.first_inp = ConvNormAct(sd, e + "first_inp.", dev, 7)
        self.first_ref = ConvNormAct(sd, e + "first_ref.", dev, 7)
        self.inp_down = [ConvNormAct(sd, f"{e}inp_down{i}.", dev, 3, pool=True) for i in range(3)]
        self.ref_down = [ConvNormAct(sd, f"{e}ref_down{i}.", dev, 3, pool=True) for i in range(3)]
        self.ca2 = Transformer(sd, e + "ca2.", dev)
        self.audio = []
        for i, (stride, pad, res) in enumerate(AUDIO_CFG):
            a = f"{p}audio_encoder.{i}.conv_block."
            self.audio.append((ConvW(sd[a + "0.weight"], sd[a + "0.bias"], dev, stride=stride, padding=pad,
                                     bn=bn_tuple(sd, a + "1.")), res))
        d = p + "decoder."
        self.bank = AdainBank(sd[f"{d}res2.res0.conv1.bn_l.mlp_shared.0.weight"].shape[1])
        self.levels = []
        chans = {2: 1024, 1: 256, 0: 128}
        sizes = {2: (12, 12), 1: (24, 24), 0: (48, 48)}
        for i in (2, 1, 0):
            blocks = []
            for j in range(9):
                r = f"{d}res{i}.res{j}."
                blocks.append((FFCLama(sd, r + "conv1.", dev, chans[i], sizes[i], self.bank),
                               FFCLama(sd, r + "conv2.", dev, chans[i], sizes[i], self.bank)))
            self.levels.append(dict(i=i, c=chans[i], blocks=blocks,
                                    up=ConvNormAct(sd, f"{d}up{i}.", dev, 3, up=True),
                                    jump=ConvNormAct(sd, f"{d}jump{i}.", dev, 3)))
        self.bank.build(dev)
        self.final = make_conv(sd, d + "final.model.0.", dev, padding=3)
        fw = conv_weight(sd, d + "final.model.0.")                 # 4-output variant (4th row zero)
        self.final4 = ConvW(torch.cat([fw, torch.zeros((1,) + tuple(fw.shape[1:]))]),
                            torch.cat([sd[d + "final.model.0.bias"].float(), torch.zeros(1)]), dev, padding=3)

    @staticmethod
    def _shape_after(layers, n, h, w):
        c = 0
        for L in layers:
            h, w = L.conv.out_hw(h, w)
            if L.pool:
                h, w = h // 2, w // 2
            c = L.conv.cout
        return n, h, w, c

    def _branches(self, ctx):
        side = ctx.streams(("lnet", id(self)), 2)
        return None if side is None else Branches(self.device, side)

    def forward(self, ctx, audio: torch.Tensor, face6: NHWC, out: NHWC, logits: NHWC | None = None,
                pad_rgb: bool = False, on_level=None):
        """audio: [B,1,80,16] device tensor; face6: NHWC [B,96,96,6] = [masked | ref];
        out: NHWC [B,96,96,3] receives sigmoid(final conv) ([B,96,96,4] with a 4th constant channel
        when ``pad_rgb``).  ``on_level(h)``: called on the calling stream before the decoder level of
        h x h starts (ENet forks its style encoder there, engine/enet.py FORK_AT)."""
        dev = self.device
        b = face6.n
        # ---- visual encoder (LNet.py:30-43) and audio encoder (LNet.py:102-120): the masked-face
        # stream, the reference stream and the audio encoder (+ the ADAIN heads it feeds) are
        # independent until the cross attention, so they run as three concurrent branches
        n_, oh, ow, c = self._shape_after([self.first_ref] + self.ref_down, b, face6.h, face6.w)
        cat = NHWC.empty(n_, oh, ow, 2 * c, dev)
        skips = []
        st = {}

        def masked(cx):
            xm = self.first_inp(cx, face6.slice(0, 3))
            skips.append(xm)
            for i in range(3):
                xm = self.inp_down[i](cx, xm)
                if i < 2:
                    skips.append(xm)
            st["xm2"] = xm

        def reference(cx):
            xr = self.first_ref(cx, face6.slice(3, 3))
            for i in range(3):
                xr = self.ref_down[i](cx, xr, out=cat.slice(c, c) if i == 2 else None)

        def audio_enc(cx):
            a = audio.contiguous()
            x = NHWC(a.view(b, a.shape[2], a.shape[3], 1))
            for cw, res in self.audio:
                oh2, ow2 = cw.out_hw(x.h, x.w)
                y = NHWC.empty(b, oh2, ow2, cw.cout, dev)
                ops.conv2d(cx, x, cw, y, act=ops.ACT_RELU, res=x if res else None)
                x = y
            st["adain"] = self.bank.run(cx, x)

        br = self._branches(ctx) if BRANCHES else None
        if br is None:
            masked(ctx)
            reference(ctx)
            audio_enc(ctx)
        else:
            fns = dict(m=masked, r=reference, a=audio_enc)
            br.run(ctx, *(fns[k] for k in ENC_ORDER))
        self.ca2(ctx, st["xm2"], cat.slice(c, c), cat.slice(0, c))
        ap = st["adain"]                                        # ADAIN gamma / beta of every FFC
        # ---- decoder (LNet.py:67-77)
        cur = cat
        for lv in self.levels:
            c = lv["c"]
            if on_level is not None:
                on_level(cur.h)
            ya = NHWC.empty(cur.n, cur.h, cur.w, c, dev)
            yb = NHWC.empty(cur.n, cur.h, cur.w, c, dev)
            # the ADAIN that ends each FFC also writes the reflect-padded copy the next FFC's 3x3
            # convs read (PREPAD), so no separate pad pass runs inside a level
            pa = pc = None
            if PREPAD and FUSED_PAD:
                pa = NHWC.empty(cur.n, cur.h + 2, cur.w + 2, c, dev)
                pc = NHWC.empty(cur.n, cur.h + 2, cur.w + 2, c, dev)
            nblk = len(lv["blocks"])
            fbr = None if GROUP else br                         # grouped FFC: one stream
            for bi, (l1, l2) in enumerate(lv["blocks"]):
                u1 = l1.pre_norm(ctx, cur, ya, fbr, xpad=pc if bi > 0 else None)
                l1.norm(ctx, self.bank, ap, ya, ya, pad_out=pa, u=u1)
                u2 = l2.pre_norm(ctx, ya, yb, fbr, xpad=pa)
                l2.norm(ctx, self.bank, ap, yb, cur, res=cur,    # FFCResnetBlock: id + conv2(conv1(x))
                        pad_out=pc if bi + 1 < nblk else None, u=u2)
            up = lv["up"](ctx, cur)
            skip = skips.pop()
            lv["jump"](ctx, skip, out=up, res=up)               # jump(skip) + out
            cur = up
        if logits is not None:
            ops.conv2d(ctx, cur, self.final, logits)
        ops.conv2d(ctx, cur, self.final4 if pad_rgb else self.final, out, act=ops.ACT_SIGMOID)
        return out
