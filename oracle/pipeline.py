"""CPU restatement of the per-frame glue around the networks (TEST INFRASTRUCTURE ONLY).

  DNet fake -> uint8 stabilised frame                 preprocessing/facing.py:189-191
  ENet inputs: [masked original | ref] / 255, gt=ref  inference.py:393-399 (img_size//2 rows masked)
  ENet output -> clamp(0, 1) * 255 -> uint8           inference.py:266-288
"""
import numpy as np
import torch

from . import nets


def to_u8_m11(x: torch.Tensor) -> torch.Tensor:
    """np.uint8((x.clamp(-1, 1) + 1) / 2 * 255) (truncation)."""
    return ((x.clamp(-1, 1) + 1) / 2 * 255).to(torch.uint8)


def lipsync_inputs(src: torch.Tensor, fake: torch.Tensor):
    ref_u8 = to_u8_m11(fake)
    orig_u8 = to_u8_m11(src)
    h = src.shape[-2]
    masked = orig_u8.clone()
    masked[:, :, h // 2:] = 0
    face6 = torch.cat([masked, ref_u8], 1).float() / 255.0
    return ref_u8, face6, ref_u8.float() / 255.0


def lipsync_frames(sd_dnet, sd_enet, mel, src, coeff):
    """mel [b,1,80,16], src [b,3,256,256] in [-1,1], coeff [b,73,26] -> uint8 [b,3,384,384]."""
    with torch.no_grad():
        fake = nets.dnet_forward(sd_dnet, src, coeff)["fake_image"]
        _, face6, gt = lipsync_inputs(src, fake)
        out, _ = nets.enet_forward(sd_enet, mel, face6, gt)
    return (out.clamp(0, 1) * 255).to(torch.uint8)
