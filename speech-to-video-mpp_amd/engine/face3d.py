"""face3d ReconNetWrapper('resnet50') engine (third_part/face3d/models/networks.py:66-105, :355-372)
on libs2v, NHWC.

  * the ResNet-50 body is the one RetinaFace uses (engine/retinaface.py ResNet50Body: every eval
    BatchNorm folded into its conv's epilogue, the bottleneck's identity add + relu fused into conv3);
  * AdaptiveAvgPool2d((1, 1)) is s2v_spatial_mean_nhwc on the [n, 7, 7, 2048] layer4 output;
  * the seven 1x1 final_layers (id | exp | tex | angle | gamma | tx,ty | tz) are ONE 2048 -> 257
    conv with the seven biases in its epilogue; torch.flatten(torch.cat(outputs, 1), 1) is that
    conv's output row.
"""
from __future__ import annotations

import torch

from .. import ops
from ..models.face3d_arch import FC_DIM, FINAL_DIMS
from ..ops import NHWC, ConvW
from .retinaface import ResNet50Body


class ReconNetEngine:
    def __init__(self, sd, device):
        dev = torch.device(device)
        self.device = dev
        self.body = ResNet50Body(sd, "backbone.", dev)
        ws = [sd[f"final_layers.{i}.weight"].float() for i in range(len(FINAL_DIMS))]
        bs = [sd[f"final_layers.{i}.bias"].float() for i in range(len(FINAL_DIMS))]
        self.head = ConvW(torch.cat(ws), torch.cat(bs), dev)

    def forward(self, ctx, x4: NHWC) -> torch.Tensor:
        """x4 [n, H, W, 4] fp32 (RGB / 255, channel 3 zero) -> coefficients [n, 257] (a view)."""
        feat = self.body(ctx, x4)[-1]
        n = feat.n
        pooled = NHWC.empty(n, 1, 1, feat.c, self.device)
        ops.check(ctx.lib.s2v_spatial_mean_nhwc(feat.ptr, n, feat.h * feat.w, feat.c, pooled.ptr, ctx.stream),
                  "s2v_spatial_mean_nhwc")
        out = NHWC.empty(n, 1, 1, (FC_DIM + 3) // 4 * 4, self.device)
        ops.conv2d(ctx, pooled, self.head, out.slice(0, FC_DIM))
        return out.t.view(n, -1)[:, :FC_DIM]
