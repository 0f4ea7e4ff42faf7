"""Parameter layout of GPEN's ParseNet face parser (third_part/GPEN/face_parse/parse_model.py:21-75,
blocks.py:8-126), as FaceParse builds it: ParseNet(512, 512, 32, 64, 19, norm_type='bn',
relu_type='LeakyReLU', ch_range=[32, 256]) (face_parsing.py:33-37).

Like ``arch``, the classes only declare parameters / buffers under the reference attribute paths,
so a ``ParseNet-latest.pth`` state_dict loads with strict=True.  Each conv layer also records the
spec the engine builds its launch from (channels, kernel, scale, norm, activation, reflect pad).
"""
from __future__ import annotations

import math

from torch import nn


class NormLayerParams(nn.Module):
    """blocks.py:8-38; only 'bn', 'gn' and 'layer' carry state ('in', 'pixel', 'none' do not)."""

    def __init__(self, channels, normalize_shape=None, norm_type="bn"):
        super().__init__()
        self.norm_type = norm_type.lower()
        if self.norm_type == "bn":
            self.norm = nn.BatchNorm2d(channels, affine=True)
        elif self.norm_type == "gn":
            self.norm = nn.GroupNorm(32, channels, affine=True)
        elif self.norm_type == "layer":
            self.norm = nn.LayerNorm(normalize_shape)
        elif self.norm_type not in ("in", "pixel", "none"):
            raise ValueError(f"Norm type {norm_type} not support.")


class ReluLayerParams(nn.Module):
    """blocks.py:41-69; PReLU is the only variant with parameters."""

    def __init__(self, channels, relu_type="relu"):
        super().__init__()
        self.relu_type = relu_type.lower()
        if self.relu_type == "prelu":
            self.func = nn.PReLU(channels)
        elif self.relu_type not in ("relu", "leakyrelu", "selu", "none"):
            raise ValueError(f"Relu type {relu_type} not support.")


class ConvLayerParams(nn.Module):
    """blocks.py:72-99: [nearest x2 if scale == 'up'] -> ReflectionPad2d(ceil((k-1)/2)) -> Conv2d
    (stride 2 if scale == 'down'; no bias under 'bn') -> norm -> activation."""

    def __init__(self, in_channels, out_channels, kernel_size=3, scale="none", norm_type="none",
                 relu_type="none", use_pad=True, bias=True):
        super().__init__()
        if norm_type in ("bn",):
            bias = False
        self.conv2d = nn.Conv2d(in_channels, out_channels, kernel_size, 2 if scale == "down" else 1, bias=bias)
        self.relu = ReluLayerParams(out_channels, relu_type)
        self.norm = NormLayerParams(out_channels, norm_type=norm_type)
        self.spec = dict(cin=in_channels, cout=out_channels, k=kernel_size,
                         scale=scale if scale in ("up", "down") else "none",
                         norm=norm_type.lower(), relu=relu_type.lower(),
                         pad=int(math.ceil((kernel_size - 1.0) / 2)) if use_pad else 0)


class ResidualBlockParams(nn.Module):
    """blocks.py:102-126: shortcut (identity when scale == 'none' and c_in == c_out, else a plain
    ConvLayer with the block's scale), conv1 (norm + act), conv2 (norm, no act)."""

    _SCALES = {"down": ("none", "down"), "up": ("up", "none"), "none": ("none", "none")}

    def __init__(self, c_in, c_out, relu_type="prelu", norm_type="bn", scale="none"):
        super().__init__()
        self.shortcut_func = None if (scale == "none" and c_in == c_out) else ConvLayerParams(c_in, c_out, 3, scale)
        s1, s2 = self._SCALES[scale]
        self.conv1 = ConvLayerParams(c_in, c_out, 3, s1, norm_type=norm_type, relu_type=relu_type)
        self.conv2 = ConvLayerParams(c_out, c_out, 3, s2, norm_type=norm_type, relu_type="none")

    def specs(self):
        return (None if self.shortcut_func is None else self.shortcut_func.spec, self.conv1.spec, self.conv2.spec)


class ParseNetParams(nn.Module):
    """parse_model.py:21-67: encoder (ConvLayer 3->base_ch + log2(in/min_feat) down blocks), body
    (res_depth blocks), decoder (log2(out/min_feat) up blocks), out_img_conv (->3),
    out_mask_conv (->parsing_ch); channels clipped to ch_range."""

    def __init__(self, in_size=128, out_size=128, min_feat_size=32, base_ch=64, parsing_ch=19, res_depth=10,
                 relu_type="prelu", norm_type="bn", ch_range=(32, 512)):
        super().__init__()
        lo, hi = ch_range
        clip = lambda c: max(lo, min(c, hi))  # noqa: E731
        min_feat_size = min(in_size, min_feat_size)
        down = int(math.log2(in_size // min_feat_size))
        up = int(math.log2(out_size // min_feat_size))
        act = dict(norm_type=norm_type, relu_type=relu_type)
        enc = [ConvLayerParams(3, base_ch, 3, 1)]          # scale=1: neither 'up' nor 'down'
        head = base_ch
        for _ in range(down):
            enc.append(ResidualBlockParams(clip(head), clip(head * 2), scale="down", **act))
            head *= 2
        body = [ResidualBlockParams(clip(head), clip(head), **act) for _ in range(res_depth)]
        dec = []
        for _ in range(up):
            dec.append(ResidualBlockParams(clip(head), clip(head // 2), scale="up", **act))
            head //= 2
        self.encoder = nn.Sequential(*enc)
        self.body = nn.Sequential(*body)
        self.decoder = nn.Sequential(*dec)
        self.out_img_conv = ConvLayerParams(clip(head), 3)
        self.out_mask_conv = ConvLayerParams(clip(head), parsing_ch)
        self.in_size, self.out_size, self.parsing_ch = in_size, out_size, parsing_ch

    def describe(self):
        """Layer plan for the engine: key prefixes and conv specs in forward order."""
        blocks = lambda name, seq, first=0: [(f"{name}.{i}.",) + m.specs()  # noqa: E731
                                             for i, m in enumerate(seq) if i >= first]
        return {"enc0": ("encoder.0.", self.encoder[0].spec),
                "down": blocks("encoder", self.encoder, 1),
                "body": blocks("body", self.body),
                "up": blocks("decoder", self.decoder),
                "out_img": ("out_img_conv.", self.out_img_conv.spec),
                "out_mask": ("out_mask_conv.", self.out_mask_conv.spec)}


def face_parse_net(size=512):
    """The FaceParse configuration (face_parsing.py:34)."""
    return dict(in_size=size, out_size=size, min_feat_size=32, base_ch=64, parsing_ch=19, norm_type="bn",
                relu_type="LeakyReLU", ch_range=(32, 256))
