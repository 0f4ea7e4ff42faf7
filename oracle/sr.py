"""CPU restatement of RealESRNet / RRDBNet (TEST INFRASTRUCTURE ONLY; see oracle/__init__).

RRDBNet.forward          third_part/GPEN/sr_model/rrdbnet_arch.py:8-116
pixel_unshuffle          third_part/GPEN/sr_model/arch_util.py:106-125
RealESRNet.process       third_part/GPEN/sr_model/real_esrnet.py:99-137 (tile_size = 0, the
                         FaceEnhancement configuration, face_enhancement.py:52-58)
RealESRNet.tile_process  real_esrnet.py:34-97

Written as functions of a state_dict (torch CPU fp32 aten ops + NumPy for the uint8 ends).
Pinned against tests/golden/rrdbnet_*.npz, produced by the reference modules themselves
(tests/golden/make_golden.py gen_rrdbnet).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def pixel_unshuffle(x, scale):
    """arch_util.py:106-125: channel index c * s^2 + i * s + j."""
    b, c, hh, hw = x.shape
    h, w = hh // scale, hw // scale
    return x.view(b, c, h, scale, w, scale).permute(0, 1, 3, 5, 2, 4).reshape(b, c * scale * scale, h, w)


def _conv(sd, p, x):
    return F.conv2d(x, sd[p + "weight"], sd[p + "bias"], 1, 1)


def _lrelu(x):
    return F.leaky_relu(x, 0.2)


def _rdb(sd, p, x):
    """ResidualDenseBlock.forward (rrdbnet_arch.py:30-37)."""
    feats = [x]
    for i in range(1, 5):
        feats.append(_lrelu(_conv(sd, f"{p}conv{i}.", torch.cat(feats, 1))))
    x5 = _conv(sd, p + "conv5.", torch.cat(feats, 1))
    return x5 * 0.2 + x


def rrdbnet_forward(sd, x, scale, num_block=None):
    """RRDBNet.forward (rrdbnet_arch.py:101-116)."""
    if num_block is None:
        num_block = 1 + max(int(k.split(".")[1]) for k in sd if k.startswith("body."))
    if scale == 2:
        feat = pixel_unshuffle(x, 2)
    elif scale == 1:
        feat = pixel_unshuffle(x, 4)
    else:
        feat = x
    feat = _conv(sd, "conv_first.", feat)
    body = feat
    for i in range(num_block):
        t = body
        for r in (1, 2, 3):
            t = _rdb(sd, f"body.{i}.rdb{r}.", t)
        body = t * 0.2 + body                      # RRDB.forward (:56-61)
    feat = feat + _conv(sd, "conv_body.", body)
    feat = _lrelu(_conv(sd, "conv_up1.", F.interpolate(feat, scale_factor=2, mode="nearest")))
    feat = _lrelu(_conv(sd, "conv_up2.", F.interpolate(feat, scale_factor=2, mode="nearest")))
    return _conv(sd, "conv_last.", _lrelu(_conv(sd, "conv_hr.", feat)))


def _mod_scale(scale):
    return {2: 2, 1: 4}.get(scale)


def sr_preprocess(img_u8, scale):
    """real_esrnet.py:100-115: uint8 HWC BGR -> float32 [1,3,H',W'] RGB / 255, reflect-padded on
    the bottom / right to a multiple of the unshuffle factor.  Returns (tensor, h_pad, w_pad)."""
    img = img_u8.astype(np.float32) / 255.
    t = torch.from_numpy(np.ascontiguousarray(np.transpose(img[:, :, [2, 1, 0]], (2, 0, 1)))).float().unsqueeze(0)
    h_pad = w_pad = 0
    m = _mod_scale(scale)
    if m is not None:
        _, _, h, w = t.shape
        h_pad = (m - h % m) if h % m else 0
        w_pad = (m - w % m) if w % m else 0
        t = F.pad(t, (0, w_pad, 0, h_pad), "reflect")
    return t, h_pad, w_pad


def sr_postprocess(output, h_pad, w_pad):
    """real_esrnet.py:125-131: crop the pad, clamp, RGB -> BGR HWC, (x * 255).round() -> uint8."""
    _, _, h, w = output.shape
    output = output[:, :, 0:h - h_pad, 0:w - w_pad]
    out = output.data.squeeze().float().cpu().clamp_(0, 1).numpy()
    out = np.transpose(out[[2, 1, 0], :, :], (1, 2, 0))
    return (out * 255.0).round().astype(np.uint8)


def tile_process(sd, img, scale, tile_size, tile_pad):
    """real_esrnet.py:34-97 (the tiled variant; the reference's own bookkeeping, restated)."""
    batch, channel, height, width = img.shape
    output = img.new_zeros((batch, channel, height * scale, width * scale))
    tiles_x, tiles_y = math.ceil(width / tile_size), math.ceil(height / tile_size)
    for y in range(tiles_y):
        for x in range(tiles_x):
            sx, sy = x * tile_size, y * tile_size
            ex, ey = min(sx + tile_size, width), min(sy + tile_size, height)
            sxp, exp_ = max(sx - tile_pad, 0), min(ex + tile_pad, width)
            syp, eyp = max(sy - tile_pad, 0), min(ey + tile_pad, height)
            tile = rrdbnet_forward(sd, img[:, :, syp:eyp, sxp:exp_], scale)
            ox, oy = (sx - sxp) * scale, (sy - syp) * scale
            output[:, :, sy * scale:ey * scale, sx * scale:ex * scale] = \
                tile[:, :, oy:oy + (ey - sy) * scale, ox:ox + (ex - sx) * scale]
    return output


def realesrnet_process(sd, img_u8, scale=2, tile_size=0, tile_pad=10):
    """RealESRNet.process (real_esrnet.py:99-137) on one uint8 BGR frame."""
    t, h_pad, w_pad = sr_preprocess(img_u8, scale)
    with torch.no_grad():
        out = tile_process(sd, t, scale, tile_size, tile_pad) if tile_size > 0 else rrdbnet_forward(sd, t, scale)
    return sr_postprocess(out, h_pad, w_pad)
