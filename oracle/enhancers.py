"""CPU restatement of the 512x512 face enhancers (TEST INFRASTRUCTURE ONLY; see oracle/__init__).

GFPGANv1Clean   third_part/GFPGAN/gfpgan/archs/gfpganv1_clean_arch.py:11-324,
                stylegan2_clean_arch.py:10-367
GPEN            third_part/GPEN/face_model/gpen_model.py:18-630, op/fused_act.py:57-96,
                op/upfirdn2d.py:149-193 (the CPU fallbacks, i.e. the reference's own oracle for its
                two CUDA kernels)

Pinned against tests/golden/gfpgan_b1_512.npz and gpen_b1_512.npz (produced by the reference
modules themselves, tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .nets import conv, linear, modulated_conv


def _lrelu(x):
    return F.leaky_relu(x, 0.2)


# ----------------------------------------------------------------------------- GFPGAN
def _resblock(sd, p, x, scale):
    """gfpganv1_clean_arch.py:131-149 (bilinear down/up ResBlock)."""
    y = _lrelu(conv(sd, p + "conv1.", x, 1, 1))
    y = F.interpolate(y, scale_factor=scale, mode="bilinear", align_corners=False)
    y = _lrelu(conv(sd, p + "conv2.", y, 1, 1))
    xs = F.interpolate(x, scale_factor=scale, mode="bilinear", align_corners=False)
    return y + F.conv2d(xs, sd[p + "skip.weight"])


def _style_conv(sd, p, x, style, sample_mode, noise):
    """stylegan2_clean_arch.py:126-138 (noise: the stored buffer, randomize_noise=False)."""
    y = modulated_conv(sd, p + "modulated_conv.", x, style, True, sample_mode) * 2 ** 0.5
    y = y + sd[p + "weight"] * noise
    return _lrelu(y + sd[p + "bias"])


def _to_rgb(sd, p, x, style, skip):
    """stylegan2_clean_arch.py:157-175."""
    y = modulated_conv(sd, p + "modulated_conv.", x, style, False, None) + sd[p + "bias"]
    if skip is not None:
        y = y + F.interpolate(skip, scale_factor=2, mode="bilinear", align_corners=False)
    return y


def gfpgan_forward(sd, x, noises=None, return_rgb=True, num_style_feat=512, sft_half=True):
    """GFPGANv1Clean.forward with input_is_latent=True, different_w=True (GFPGANer's build).
    ``noises``: per-layer [B|1,1,H,W] tensors, default the stored buffers."""
    log_size = int(math.log2(x.shape[-1]))
    b = x.shape[0]
    feat = _lrelu(conv(sd, "conv_body_first.", x))
    skips = []
    for i in range(log_size - 2):
        feat = _resblock(sd, f"conv_body_down.{i}.", feat, 0.5)
        skips.insert(0, feat)
    feat = _lrelu(conv(sd, "final_conv.", feat, 1, 1))
    style = linear(sd, "final_linear.", feat.reshape(b, -1)).reshape(b, -1, num_style_feat)
    conditions, rgbs = [], []
    for i in range(log_size - 2):
        feat = _resblock(sd, f"conv_body_up.{i}.", feat + skips[i], 2)
        for branch in ("condition_scale", "condition_shift"):
            q = f"{branch}.{i}."
            conditions.append(conv(sd, q + "2.", _lrelu(conv(sd, q + "0.", feat, 1, 1)), 1, 1))
        if return_rgb:
            rgbs.append(conv(sd, f"toRGB.{i}.", feat))
    d = "stylegan_decoder."
    nl = (log_size - 2) * 2 + 1
    if noises is None:
        noises = [sd[f"{d}noises.noise{i}"] for i in range(nl)]
    out = sd[d + "constant_input.weight"].repeat(b, 1, 1, 1)
    out = _style_conv(sd, d + "style_conv1.", out, style[:, 0], None, noises[0])
    skip = _to_rgb(sd, d + "to_rgb1.", out, style[:, 1], None)
    i = 1
    for lvl in range(log_size - 2):
        out = _style_conv(sd, f"{d}style_convs.{2 * lvl}.", out, style[:, i], "upsample", noises[2 * lvl + 1])
        if i < len(conditions):                             # gfpganv1_clean_arch.py:103-112
            if sft_half:
                c = out.shape[1] // 2
                out = torch.cat([out[:, :c], out[:, c:] * conditions[i - 1] + conditions[i]], 1)
            else:
                out = out * conditions[i - 1] + conditions[i]
        out = _style_conv(sd, f"{d}style_convs.{2 * lvl + 1}.", out, style[:, i + 1], None, noises[2 * lvl + 2])
        skip = _to_rgb(sd, f"{d}to_rgbs.{lvl}.", out, style[:, i + 2], skip)
        i += 2
    return skip, rgbs, style


# ----------------------------------------------------------------------------- GPEN
def upfirdn2d(x, kernel, up=1, down=1, pad=(0, 0)):
    """op/upfirdn2d.py:149-193 (upfirdn2d_native, symmetric pads)."""
    b, c, h, w = x.shape
    kh, kw = kernel.shape
    p0, p1 = pad
    y = x.reshape(b * c, h, 1, w, 1)
    y = F.pad(y, [0, up - 1, 0, 0, 0, up - 1]).reshape(b * c, 1, h * up, w * up)
    y = F.pad(y, [max(p0, 0), max(p1, 0), max(p0, 0), max(p1, 0)])
    y = y[:, :, max(-p0, 0): y.shape[2] - max(-p1, 0), max(-p0, 0): y.shape[3] - max(-p1, 0)]
    y = F.conv2d(y, torch.flip(kernel, [0, 1]).reshape(1, 1, kh, kw))
    return y.reshape(b, c, y.shape[-2], y.shape[-1])[:, :, ::down, ::down]


def fused_leaky_relu(x, bias, slope=0.2, scale=2 ** 0.5):
    """op/fused_act.py:92-96 (CPU form)."""
    return scale * F.leaky_relu(x + bias.reshape((1, -1) + (1,) * (x.dim() - 2)), slope)


def _equal_linear(sd, p, x, lr_mul=1.0, act=False):
    """gpen_model.py:149-162."""
    w = sd[p + "weight"]
    y = F.linear(x, w * (lr_mul / math.sqrt(w.shape[1])))
    if act:
        return fused_leaky_relu(y, sd[p + "bias"] * lr_mul)
    return y + sd[p + "bias"] * lr_mul


def _conv_layer(sd, p, x, k, downsample):
    """gpen_model.py:515-562 ConvLayer (activate=True, bias=True)."""
    i = 0
    if downsample:
        x = upfirdn2d(x, sd[p + "0.kernel"], pad=(2, 2))    # p = (4-2)+(3-1) = 4 -> (2, 2)
        i = 1
    w = sd[f"{p}{i}.weight"]
    x = F.conv2d(x, w * (1 / math.sqrt(w[0].numel())), stride=2 if downsample else 1,
                 padding=0 if downsample else k // 2)
    return fused_leaky_relu(x, sd[f"{p}{i + 1}.bias"])


def _gpen_modconv(sd, p, x, style, demodulate=True, upsample=False):
    """gpen_model.py:245-290."""
    b, cin, h, w = x.shape
    wt = sd[p + "weight"]
    o, k = wt.shape[1], wt.shape[-1]
    s = _equal_linear(sd, p + "modulation.", style).reshape(b, 1, cin, 1, 1)
    wt = wt * (1 / math.sqrt(cin * k * k)) * s
    if demodulate:
        wt = wt * torch.rsqrt(wt.pow(2).sum([2, 3, 4]) + 1e-8).reshape(b, o, 1, 1, 1)
    if upsample:
        wt = wt.transpose(1, 2).reshape(b * cin, o, k, k)
        y = F.conv_transpose2d(x.reshape(1, b * cin, h, w), wt, padding=0, stride=2, groups=b)
        y = y.reshape(b, o, y.shape[-2], y.shape[-1])
        return upfirdn2d(y, sd[p + "blur.kernel"], pad=(1, 1))  # p=0 -> (0+1, 0+1)
    y = F.conv2d(x.reshape(1, b * cin, h, w), wt.reshape(b * o, cin, k, k), padding=k // 2, groups=b)
    return y.reshape(b, o, h, w)


def _styled_conv(sd, p, x, style, noise, upsample=False):
    """gpen_model.py:353-363 (NoiseInjection isconcat: cat(out, w * noise))."""
    y = _gpen_modconv(sd, p + "conv.", x, style, True, upsample)
    y = torch.cat([y, sd[p + "noise.weight"] * noise], 1)
    return fused_leaky_relu(y, sd[p + "activate.bias"])


def _gpen_to_rgb(sd, p, x, style, skip):
    """gpen_model.py:374-384."""
    y = _gpen_modconv(sd, p + "conv.", x, style, False) + sd[p + "bias"]
    if skip is not None:
        y = y + upfirdn2d(skip, sd[p + "upsample.kernel"], up=2, pad=(2, 1))
    return y


def gpen_forward(sd, x, n_mlp=8, lr_mlp=0.01):
    """FullGenerator.forward (gpen_model.py:608-630) -> (image, latent)."""
    log_size = int(math.log2(x.shape[-1]))
    feats = []
    h = x
    for i in range(log_size - 1):
        h = _conv_layer(sd, f"ecd{i}.0.", h, 1 if i == 0 else 3, downsample=i > 0)
        feats.append(h)
    code = _equal_linear(sd, "final_linear.0.", h.reshape(h.shape[0], -1), act=True)
    noise = [f for f in feats[::-1] for _ in range(2)][1:]   # repeat x2, reversed, drop first
    g = "generator."
    lat = code * torch.rsqrt(torch.mean(code ** 2, dim=1, keepdim=True) + 1e-8)   # PixelNorm
    for i in range(1, n_mlp + 1):
        lat = _equal_linear(sd, f"{g}style.{i}.", lat, lr_mul=lr_mlp, act=True)
    b = x.shape[0]
    out = sd[g + "input.input"].repeat(b, 1, 1, 1)
    out = _styled_conv(sd, g + "conv1.", out, lat, noise[0])
    skip = _gpen_to_rgb(sd, g + "to_rgb1.", out, lat, None)
    for lvl in range(log_size - 2):
        out = _styled_conv(sd, f"{g}convs.{2 * lvl}.", out, lat, noise[2 * lvl + 1], upsample=True)
        out = _styled_conv(sd, f"{g}convs.{2 * lvl + 1}.", out, lat, noise[2 * lvl + 2])
        skip = _gpen_to_rgb(sd, f"{g}to_rgbs.{lvl}.", out, lat, skip)
    return skip, lat, code
