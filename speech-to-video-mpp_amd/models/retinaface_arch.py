"""Parameter layout of GPEN's RetinaFace-R50 face detector (third_part/GPEN/face_detect/facemodels/
retinaface.py:47-125, net.py:8-100, data/config.py cfg_re50), as RetinaFaceDetection builds it
(face_detect/retinaface_detection.py:19-30): RetinaFace(cfg=cfg_re50, phase='test').

The backbone is torchvision's resnet50 cut by IntermediateLayerGetter at layer2 / layer3 / layer4
(``body.*`` keys: conv1, bn1, layer1..4 of Bottleneck blocks [3, 4, 6, 3], expansion 4, the stride
on conv2 of the first block of layers 2-4, a 1x1 + BN ``downsample`` on every first block); then
the FPN (1x1 lateral conv_bn1X1 + 3x3 merge conv_bn, leaky 0 since out_channel 256 > 64), three
SSH context modules and the per-level 1x1 class / box / landmark heads (2 anchors each).  The
classes only declare parameters / buffers under the reference attribute paths, so a
``RetinaFace-R50.pth`` state_dict (``module.`` prefix stripped) loads with strict=True.
"""
from __future__ import annotations

from torch import nn

CFG_RE50 = dict(name="Resnet50", min_sizes=[[16, 32], [64, 128], [256, 512]], steps=[8, 16, 32],
                variance=[0.1, 0.2], clip=False, return_layers={"layer2": 1, "layer3": 2, "layer4": 3},
                in_channel=256, out_channel=256)     # data/config.py:22-41 (inference fields)


def _conv_bn(cin, cout, k, stride=1):
    """net.py conv_bn / conv_bn_no_relu / conv_bn1X1: Conv2d(bias=False) -> BatchNorm2d [-> LeakyReLU]."""
    return nn.Sequential(nn.Conv2d(cin, cout, k, stride, k // 2, bias=False), nn.BatchNorm2d(cout))


class BottleneckParams(nn.Module):
    """torchvision.models.resnet.Bottleneck (v1.5: stride on the 3x3 conv)."""

    def __init__(self, inplanes, planes, stride=1, downsample=False):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.stride = stride
        if downsample:
            self.downsample = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride, bias=False),
                                            nn.BatchNorm2d(planes * 4))


class ResNet50BodyParams(nn.Module):
    """IntermediateLayerGetter(resnet50, {'layer2', 'layer3', 'layer4'}): conv1 .. layer4."""

    LAYERS = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))

    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        inplanes = 64
        for li, (planes, blocks, stride) in enumerate(self.LAYERS):
            mods = [BottleneckParams(inplanes, planes, stride, downsample=True)]
            inplanes = planes * 4
            mods += [BottleneckParams(inplanes, planes) for _ in range(blocks - 1)]
            setattr(self, f"layer{li + 1}", nn.Sequential(*mods))


class SSHParams(nn.Module):
    """net.py:38-66 SSH(256, 256)."""

    def __init__(self, cin, cout):
        super().__init__()
        self.conv3X3 = _conv_bn(cin, cout // 2, 3)
        self.conv5X5_1 = _conv_bn(cin, cout // 4, 3)
        self.conv5X5_2 = _conv_bn(cout // 4, cout // 4, 3)
        self.conv7X7_2 = _conv_bn(cout // 4, cout // 4, 3)
        self.conv7x7_3 = _conv_bn(cout // 4, cout // 4, 3)


class FPNParams(nn.Module):
    """net.py:68-100 FPN([512, 1024, 2048], 256)."""

    def __init__(self, cins, cout):
        super().__init__()
        self.output1 = _conv_bn(cins[0], cout, 1)
        self.output2 = _conv_bn(cins[1], cout, 1)
        self.output3 = _conv_bn(cins[2], cout, 1)
        self.merge1 = _conv_bn(cout, cout, 3)
        self.merge2 = _conv_bn(cout, cout, 3)


class _Head(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv1x1 = nn.Conv2d(cin, cout, 1)


class RetinaFaceParams(nn.Module):
    """retinaface.py:47-125 with cfg_re50."""

    def __init__(self, cfg=CFG_RE50):
        super().__init__()
        self.cfg = dict(cfg)
        self.body = ResNet50BodyParams()
        c = cfg["in_channel"]
        oc = cfg["out_channel"]
        self.fpn = FPNParams([c * 2, c * 4, c * 8], oc)
        self.ssh1, self.ssh2, self.ssh3 = SSHParams(oc, oc), SSHParams(oc, oc), SSHParams(oc, oc)
        self.ClassHead = nn.ModuleList([_Head(oc, 2 * 2) for _ in range(3)])
        self.BboxHead = nn.ModuleList([_Head(oc, 2 * 4) for _ in range(3)])
        self.LandmarkHead = nn.ModuleList([_Head(oc, 2 * 10) for _ in range(3)])
