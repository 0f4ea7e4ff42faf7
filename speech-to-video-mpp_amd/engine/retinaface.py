"""RetinaFace-R50 engine (third_part/GPEN/face_detect/facemodels/retinaface.py:47-125, net.py:40-100,
torchvision resnet50 as IntermediateLayerGetter layer2..4), NHWC on libs2v.

Every conv is one s2v_conv2d launch with its eval BatchNorm folded into the epilogue:
  * ResNet-50 Bottleneck: 1x1 (relu) -> 3x3 stride s (relu) -> 1x1 whose epilogue adds the
    identity (or the 1x1 stride-s downsample conv's output) before the relu; the stem is the 7x7
    stride-2 conv on the 4-channel NHWC input (BGR minus means, channel 3 zero), then
    s2v_maxpool2d_nhwc (3, 2, 1);
  * FPN: the lateral 1x1 convs (relu, leaky 0 at 256 channels) add the nearest-upsampled coarser
    level in their epilogue (residual after the activation), then the 3x3 merge convs;
  * SSH: conv3X3 and conv5X5_1 read the same input and run as ONE 256 -> 192 conv; the final
    relu(cat) is applied per branch in each conv's epilogue (relu(cat(a, b, c)) = cat(relu a, ..)),
    so the branches are written straight into one 320-channel buffer laid out
    [conv5X5_1 (64) | conv3X3 (128) | conv5X5 (64) | conv7X7 (64)]; the heads read channels
    [64, 320), i.e. exactly cat(conv3X3, conv5X5, conv7X7);
  * the three per-level heads (BboxHead 8, ClassHead 4, LandmarkHead 20 channels) are ONE 1x1 conv
    256 -> 32 per level; s2v_retina_decode reads that layout (softmax, priors, decode, threshold).
"""
from __future__ import annotations

import torch

from .. import ops
from ..ops import NHWC, ConvW

RELU = ops.ACT_RELU


def _bn(sd, p):
    return tuple(sd[p + k].float() for k in ("weight", "bias", "running_mean", "running_var"))


def _cat_bn(*bns):
    return tuple(torch.cat([b[i] for b in bns]) for i in range(4))


class _Bottleneck:
    def __init__(self, sd, p, stride, dev):
        self.c1 = ConvW(sd[p + "conv1.weight"], None, dev, bn=_bn(sd, p + "bn1."))
        self.c2 = ConvW(sd[p + "conv2.weight"], None, dev, stride=stride, padding=1, bn=_bn(sd, p + "bn2."))
        self.c3 = ConvW(sd[p + "conv3.weight"], None, dev, bn=_bn(sd, p + "bn3."))
        self.ds = None
        if p + "downsample.0.weight" in sd:
            self.ds = ConvW(sd[p + "downsample.0.weight"], None, dev, stride=stride, bn=_bn(sd, p + "downsample.1."))

    def __call__(self, ctx, x: NHWC) -> NHWC:
        dev = x.t.device
        t1 = NHWC.empty(x.n, x.h, x.w, self.c1.cout, dev)
        ops.conv2d(ctx, x, self.c1, t1, act=RELU)
        oh, ow = self.c2.out_hw(x.h, x.w)
        t2 = NHWC.empty(x.n, oh, ow, self.c2.cout, dev)
        ops.conv2d(ctx, t1, self.c2, t2, act=RELU)
        idn = x
        if self.ds is not None:
            idn = NHWC.empty(x.n, oh, ow, self.ds.cout, dev)
            ops.conv2d(ctx, x, self.ds, idn)
        y = NHWC.empty(x.n, oh, ow, self.c3.cout, dev)
        ops.conv2d(ctx, t2, self.c3, y, act=RELU, res=idn)
        return y


class _SSH:
    def __init__(self, sd, p, dev):
        def w(name):
            return sd[p + name + ".0.weight"]
        self.a = ConvW(torch.cat([w("conv5X5_1"), w("conv3X3")]), None, dev, padding=1,
                       bn=_cat_bn(_bn(sd, p + "conv5X5_1.1."), _bn(sd, p + "conv3X3.1.")))
        self.c5 = ConvW(w("conv5X5_2"), None, dev, padding=1, bn=_bn(sd, p + "conv5X5_2.1."))
        self.c72 = ConvW(w("conv7X7_2"), None, dev, padding=1, bn=_bn(sd, p + "conv7X7_2.1."))
        self.c73 = ConvW(w("conv7x7_3"), None, dev, padding=1, bn=_bn(sd, p + "conv7x7_3.1."))

    def __call__(self, ctx, x: NHWC) -> NHWC:
        """-> [n, h, w, 320] buffer; channels [64, 320) are relu(cat(conv3X3, conv5X5, conv7X7))."""
        dev = x.t.device
        o = NHWC.empty(x.n, x.h, x.w, 320, dev)
        ops.conv2d(ctx, x, self.a, o.slice(0, 192), act=RELU)
        c51 = o.slice(0, 64)
        ops.conv2d(ctx, c51, self.c5, o.slice(192, 64), act=RELU)
        t = NHWC.empty(x.n, x.h, x.w, 64, dev)
        ops.conv2d(ctx, c51, self.c72, t, act=RELU)
        ops.conv2d(ctx, t, self.c73, o.slice(256, 64), act=RELU)
        return o


class ResNet50Body:
    """torchvision resnet50 conv1 .. layer4 (Bottleneck v1.5, [3, 4, 6, 3]) with its parameters
    under ``prefix``: RetinaFace's ``body.`` (IntermediateLayerGetter) and face3d ReconNet's
    ``backbone.`` (models/networks.py:226-372, the same torchvision layout)."""
    LAYERS = ((3, 1), (4, 2), (6, 2), (3, 2))

    def __init__(self, sd, prefix, dev):
        b = prefix
        self.stem = ConvW(ops.pad_cin(sd[b + "conv1.weight"].float(), 4), None, dev, stride=2, padding=3,
                          bn=_bn(sd, b + "bn1."))
        self.layers = []
        for li, (blocks, stride) in enumerate(self.LAYERS):
            self.layers.append([_Bottleneck(sd, f"{b}layer{li + 1}.{j}.", stride if j == 0 else 1, dev)
                                for j in range(blocks)])

    def __call__(self, ctx, x4: NHWC):
        """x4 [n,H,W,4] (channel 3 zero) -> (layer1, layer2, layer3, layer4) outputs."""
        dev = x4.t.device
        oh, ow = self.stem.out_hw(x4.h, x4.w)
        s = NHWC.empty(x4.n, oh, ow, 64, dev)
        ops.conv2d(ctx, x4, self.stem, s, act=RELU)
        ph, pw = (oh + 2 - 3) // 2 + 1, (ow + 2 - 3) // 2 + 1
        y = NHWC.empty(x4.n, ph, pw, 64, dev)
        ops.check(ctx.lib.s2v_maxpool2d_nhwc(s.ptr, s.n, s.h, s.w, 64, 3, 2, 1, y.ptr, ph, pw, ctx.stream),
                  "s2v_maxpool2d_nhwc")
        outs = []
        for blocks in self.layers:
            for blk in blocks:
                y = blk(ctx, y)
            outs.append(y)
        return outs


class RetinaFaceEngine:
    HEAD_CS = 32

    def __init__(self, sd, device):
        dev = torch.device(device)
        self.device = dev
        self.body = ResNet50Body(sd, "body.", dev)
        f = "fpn."
        self.out = [ConvW(sd[f"{f}output{i}.0.weight"], None, dev, bn=_bn(sd, f"{f}output{i}.1.")) for i in (1, 2, 3)]
        self.merge1 = ConvW(sd[f + "merge1.0.weight"], None, dev, padding=1, bn=_bn(sd, f + "merge1.1."))
        self.merge2 = ConvW(sd[f + "merge2.0.weight"], None, dev, padding=1, bn=_bn(sd, f + "merge2.1."))
        self.ssh = [_SSH(sd, f"ssh{i}.", dev) for i in (1, 2, 3)]
        self.heads = []
        for i in range(3):
            ws = [sd[f"{h}.{i}.conv1x1.weight"] for h in ("BboxHead", "ClassHead", "LandmarkHead")]
            bs = [sd[f"{h}.{i}.conv1x1.bias"] for h in ("BboxHead", "ClassHead", "LandmarkHead")]
            self.heads.append(ConvW(torch.cat(ws), torch.cat(bs), dev))

    def _up_add(self, ctx, coarse: NHWC, lat: ConvW, x: NHWC) -> NHWC:
        """lateral(x) + F.interpolate(coarse, size=lateral's size, mode='nearest') (net.py:87-93)."""
        dev = x.t.device
        up = NHWC.empty(x.n, x.h, x.w, coarse.c, dev)
        ops.resize_nhwc(ctx, coarse, up, mode=1)
        y = NHWC.empty(x.n, x.h, x.w, lat.cout, dev)
        ops.conv2d(ctx, x, lat, y, act=RELU, res=up, res_after=True)
        return y

    def backbone(self, ctx, x4: NHWC):
        """x4 [n,H,W,4] (BGR minus means, channel 3 zero) -> (layer2, layer3, layer4) outputs."""
        return self.body(ctx, x4)[1:]

    def fpn(self, ctx, feats):
        """net.py:79-100 -> [output1, output2, output3]."""
        dev = feats[0].t.device
        f3 = feats[2]
        o3 = NHWC.empty(f3.n, f3.h, f3.w, 256, dev)
        ops.conv2d(ctx, f3, self.out[2], o3, act=RELU)
        o2 = self._up_add(ctx, o3, self.out[1], feats[1])
        m2 = NHWC.empty(o2.n, o2.h, o2.w, 256, dev)
        ops.conv2d(ctx, o2, self.merge2, m2, act=RELU)
        o1 = self._up_add(ctx, m2, self.out[0], feats[0])
        m1 = NHWC.empty(o1.n, o1.h, o1.w, 256, dev)
        ops.conv2d(ctx, o1, self.merge1, m1, act=RELU)
        return [m1, m2, o3]

    def head_maps(self, ctx, fpn_out):
        """SSH + fused heads per level -> [n, h_l, w_l, 32] maps (box 8 | class 4 | landmarks 20)."""
        outs = []
        for i, f in enumerate(fpn_out):
            o = self.ssh[i](ctx, f)
            h = NHWC.empty(f.n, f.h, f.w, self.HEAD_CS, f.t.device)
            ops.conv2d(ctx, o.slice(64, 256), self.heads[i], h)
            outs.append(h)
        return outs

    def forward_maps(self, ctx, x4: NHWC):
        return self.head_maps(ctx, self.fpn(ctx, self.backbone(ctx, x4)))

    @staticmethod
    def split_heads(maps):
        """Head maps -> the reference's (loc [n,P,4], conf logits [n,P,2], landms [n,P,10]) (views
        concatenated over levels: retinaface.py:115-117 before the softmax)."""
        n = maps[0].n
        locs, confs, lms = [], [], []
        for m in maps:
            t = m.t.view(n, m.h * m.w, 32)
            locs.append(t[:, :, 0:8].reshape(n, -1, 4))
            confs.append(t[:, :, 8:12].reshape(n, -1, 2))
            lms.append(t[:, :, 12:32].reshape(n, -1, 10))
        return torch.cat(locs, 1), torch.cat(confs, 1), torch.cat(lms, 1)
