"""CPU restatement of GPEN's ParseNet face parser (TEST INFRASTRUCTURE ONLY; see oracle/__init__).

third_part/GPEN/face_parse/parse_model.py:69-75 (ParseNet.forward) and blocks.py:72-126
(ConvLayer, ResidualBlock) as functions of a reference-layout state_dict, torch CPU fp32 aten ops.
Pinned by tests/golden/parsenet_*.npz (the reference module itself, tests/golden/make_golden.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .nets import bn_eval


def conv_layer(sd, p, x, k=3, scale="none", norm="none", relu="none"):
    """blocks.py:92-99: [nearest x2] -> ReflectionPad2d(ceil((k-1)/2)) -> conv -> norm -> act."""
    if scale == "up":
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    pad = k // 2
    if pad:
        x = F.pad(x, (pad,) * 4, mode="reflect")
    x = F.conv2d(x, sd[p + "conv2d.weight"], sd.get(p + "conv2d.bias"), 2 if scale == "down" else 1)
    if norm == "bn":
        x = bn_eval(sd, p + "norm.norm.", x)
    if relu == "leakyrelu":
        x = F.leaky_relu(x, 0.2)
    elif relu == "relu":
        x = F.relu(x)
    elif relu == "prelu":
        x = F.prelu(x, sd[p + "relu.func.weight"])
    return x


def residual_block(sd, p, x, scale, norm="bn", relu="leakyrelu"):
    """blocks.py:120-125: shortcut(x) + conv2(conv1(x))."""
    sc = x if (p + "shortcut_func.conv2d.weight") not in sd else conv_layer(sd, p + "shortcut_func.", x, 3, scale)
    s1, s2 = {"down": ("none", "down"), "up": ("up", "none"), "none": ("none", "none")}[scale]
    r = conv_layer(sd, p + "conv1.", x, 3, s1, norm, relu)
    r = conv_layer(sd, p + "conv2.", r, 3, s2, norm, "none")
    return sc + r


def _indices(sd, prefix):
    return sorted({int(k[len(prefix):].split(".")[0]) for k in sd if k.startswith(prefix)})


def parsenet_forward(sd, x, norm="bn", relu="leakyrelu"):
    """parse_model.py:69-75 -> (out_mask, out_img)."""
    f = conv_layer(sd, "encoder.0.", x)
    for i in _indices(sd, "encoder.")[1:]:
        f = residual_block(sd, f"encoder.{i}.", f, "down", norm, relu)
    h = f
    for i in _indices(sd, "body."):
        h = residual_block(sd, f"body.{i}.", h, "none", norm, relu)
    h = f + h
    for i in _indices(sd, "decoder."):
        h = residual_block(sd, f"decoder.{i}.", h, "up", norm, relu)
    return conv_layer(sd, "out_mask_conv.", h), conv_layer(sd, "out_img_conv.", h)


@torch.no_grad()
def mask_logits(sd, img_u8_bgr):
    """FaceParse.process (face_parsing.py:39-45) after its cv2.resize: img2tensor -> ParseNet."""
    from . import post
    return parsenet_forward(sd, torch.from_numpy(post.img2tensor(img_u8_bgr)))[0]
