"""Parameter layout of face3d's 3DMM coefficient regressor (third_part/face3d/models/networks.py:
61-105 ReconNetWrapper, :226-372 ResNet, resnet50 = Bottleneck [3, 4, 6, 3]) as
futils/inference_utils.py:261-267 load_face3d_net builds it:
``define_net_recon(net_recon='resnet50', use_last_fc=False, init_path='')``.

``backbone.*`` is torchvision's resnet50 layout without ``fc`` (use_last_fc=False), followed by the
seven 1x1 ``final_layers`` (id 80 | exp 64 | tex 80 | angle 3 | gamma 27 | tx,ty 2 | tz 1 = 257
outputs).  The classes only declare parameters / buffers under the reference attribute paths, so
the ``checkpoint['net_recon']`` state_dict loads with strict=True.
"""
from __future__ import annotations

from torch import nn

from .retinaface_arch import ResNet50BodyParams

FINAL_DIMS = (80, 64, 80, 3, 27, 2, 1)     # networks.py:86-94
FC_DIM = 257


class ReconNetWrapperParams(nn.Module):
    """networks.py:66-96 with net_recon='resnet50', use_last_fc=False."""
    fc_dim = FC_DIM

    def __init__(self, net_recon="resnet50", use_last_fc=False, init_path=None):
        super().__init__()
        if net_recon != "resnet50":
            raise NotImplementedError(f"ReconNetWrapper: only resnet50 is on the inference path, got {net_recon!r}")
        if use_last_fc:
            raise NotImplementedError("ReconNetWrapper: use_last_fc=True is a training-time variant")
        self.use_last_fc = use_last_fc
        self.backbone = ResNet50BodyParams()
        self.final_layers = nn.ModuleList([nn.Conv2d(2048, d, 1, bias=True) for d in FINAL_DIMS])
