"""Parameter layouts of the two 512x512 face enhancers.

Like ``arch``, these only declare parameters / buffers under the reference attribute paths, so a
reference checkpoint (``params_ema`` for GFPGAN, the GPEN ``.pth``) loads with strict=True.

  GFPGANv1Clean   third_part/GFPGAN/gfpgan/archs/gfpganv1_clean_arch.py:11-324,
                  stylegan2_clean_arch.py:10-367
  FullGenerator   third_part/GPEN/face_model/gpen_model.py:18-630 (GPEN-BFR-512)
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .arch import ResBlockParams, StyleConvParams, ToRGBParams


def stylegan_channels(channel_multiplier=2, narrow=1.0):
    """stylegan2_clean_arch.py:209-219 / gpen_model.py:352-363 channel table (int keys)."""
    base = {4: 512, 8: 512, 16: 512, 32: 512, 64: 256 * channel_multiplier, 128: 128 * channel_multiplier,
            256: 64 * channel_multiplier, 512: 32 * channel_multiplier, 1024: 16 * channel_multiplier,
            2048: 8 * channel_multiplier}
    return {k: int(v * narrow) for k, v in base.items()}


# ----------------------------------------------------------------------------- GFPGAN (clean)
class _ConstantInput(nn.Module):
    def __init__(self, c, size=4):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(1, c, size, size))


class _SFTBranch(nn.Sequential):
    """gfpganv1_clean_arch.py:251-258: conv3x3 -> LeakyReLU(0.2) -> conv3x3."""

    def __init__(self, c, cout):
        super().__init__(nn.Conv2d(c, c, 3, 1, 1), nn.LeakyReLU(0.2, True), nn.Conv2d(c, cout, 3, 1, 1))


class StyleGAN2GeneratorCSFTParams(nn.Module):
    """stylegan2_clean_arch.py:185-262 (+ the CSFT subclass, gfpganv1_clean_arch.py:11-33)."""

    def __init__(self, out_size, num_style_feat=512, num_mlp=8, channel_multiplier=2, narrow=1, sft_half=False):
        super().__init__()
        self.num_style_feat, self.sft_half = num_style_feat, sft_half
        layers = [nn.Identity()]                           # NormStyleCode (no parameters)
        for _ in range(num_mlp):
            layers += [nn.Linear(num_style_feat, num_style_feat), nn.LeakyReLU(0.2, True)]
        self.style_mlp = nn.Sequential(*layers)
        ch = stylegan_channels(channel_multiplier, narrow)
        self.channels = ch
        self.constant_input = _ConstantInput(ch[4])
        self.style_conv1 = StyleConvParams(ch[4], ch[4], 3, num_style_feat, True, None)
        self.to_rgb1 = ToRGBParams(ch[4], num_style_feat, upsample=False)
        self.log_size = int(math.log(out_size, 2))
        self.num_layers = (self.log_size - 2) * 2 + 1
        self.num_latent = self.log_size * 2 - 2
        self.style_convs = nn.ModuleList()
        self.to_rgbs = nn.ModuleList()
        self.noises = nn.Module()
        for i in range(self.num_layers):
            r = 2 ** ((i + 5) // 2)
            self.noises.register_buffer(f"noise{i}", torch.zeros(1, 1, r, r))
        cin = ch[4]
        for i in range(3, self.log_size + 1):
            cout = ch[2 ** i]
            self.style_convs.append(StyleConvParams(cin, cout, 3, num_style_feat, True, "upsample"))
            self.style_convs.append(StyleConvParams(cout, cout, 3, num_style_feat, True, None))
            self.to_rgbs.append(ToRGBParams(cout, num_style_feat, upsample=True))
            cin = cout


class GFPGANv1CleanParams(nn.Module):
    """gfpganv1_clean_arch.py:154-260.  GFPGANer builds it with out_size=512, channel_multiplier=2,
    different_w=True, input_is_latent=True, sft_half=True (gfpgan/utils.py:40-50)."""

    def __init__(self, out_size=512, num_style_feat=512, channel_multiplier=1, decoder_load_path=None,
                 fix_decoder=True, num_mlp=8, input_is_latent=False, different_w=False, narrow=1, sft_half=False):
        super().__init__()
        if decoder_load_path:
            raise NotImplementedError("decoder_load_path: load the full GFPGAN checkpoint instead")
        self.out_size, self.input_is_latent, self.different_w = out_size, input_is_latent, different_w
        self.num_style_feat, self.sft_half = num_style_feat, sft_half
        ch = stylegan_channels(channel_multiplier, narrow * 0.5)
        self.unet_channels = ch
        self.log_size = int(math.log(out_size, 2))
        first = 2 ** self.log_size
        self.conv_body_first = nn.Conv2d(3, ch[first], 1)
        self.conv_body_down = nn.ModuleList()
        cin = ch[first]
        for i in range(self.log_size, 2, -1):
            cout = ch[2 ** (i - 1)]
            self.conv_body_down.append(ResBlockParams(cin, cout))
            cin = cout
        self.final_conv = nn.Conv2d(cin, ch[4], 3, 1, 1)
        cin = ch[4]
        self.conv_body_up = nn.ModuleList()
        for i in range(3, self.log_size + 1):
            cout = ch[2 ** i]
            self.conv_body_up.append(ResBlockParams(cin, cout))     # mode='up': same parameters
            cin = cout
        self.toRGB = nn.ModuleList([nn.Conv2d(ch[2 ** i], 3, 1) for i in range(3, self.log_size + 1)])
        lin_out = (self.log_size * 2 - 2) * num_style_feat if different_w else num_style_feat
        self.final_linear = nn.Linear(ch[4] * 4 * 4, lin_out)
        self.stylegan_decoder = StyleGAN2GeneratorCSFTParams(out_size, num_style_feat, num_mlp, channel_multiplier,
                                                             narrow, sft_half)
        self.condition_scale = nn.ModuleList()
        self.condition_shift = nn.ModuleList()
        for i in range(3, self.log_size + 1):
            c = ch[2 ** i]
            sft_out = c if sft_half else 2 * c
            self.condition_scale.append(_SFTBranch(c, sft_out))
            self.condition_shift.append(_SFTBranch(c, sft_out))


# ----------------------------------------------------------------------------- GPEN
def _blur_kernel(k=(1, 3, 3, 1), factor=1):
    """gpen_model.py:26-35 make_kernel (x factor^2 for the upsampling blurs)."""
    t = torch.tensor(k, dtype=torch.float32)
    t = t[None, :] * t[:, None]
    return t / t.sum() * (factor ** 2)


class _Blur(nn.Module):
    def __init__(self, factor=1):
        super().__init__()
        self.register_buffer("kernel", _blur_kernel(factor=factor))


class _Upsample(nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("kernel", _blur_kernel(factor=2))


class EqualConv2dParams(nn.Module):
    """gpen_model.py:94-128 (runtime scale 1/sqrt(fan_in))."""

    def __init__(self, cin, cout, k, stride=1, padding=0, bias=True):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(cout, cin, k, k))
        self.scale = 1 / math.sqrt(cin * k * k)
        self.stride, self.padding = stride, padding
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None


class EqualLinearParams(nn.Module):
    """gpen_model.py:131-167 (runtime scale lr_mul/sqrt(in), bias * lr_mul)."""

    def __init__(self, din, dout, bias=True, bias_init=0, lr_mul=1, activation=None):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(dout, din))
        self.bias = nn.Parameter(torch.full((dout,), float(bias_init))) if bias else None
        self.activation, self.lr_mul = activation, lr_mul
        self.scale = lr_mul / math.sqrt(din)


class FusedLeakyReLUParams(nn.Module):
    """op/fused_act.py:73-86: bias [C], negative_slope 0.2, scale sqrt(2)."""

    def __init__(self, c):
        super().__init__()
        self.bias = nn.Parameter(torch.zeros(c))


class GPENModulatedConv2dParams(nn.Module):
    """gpen_model.py:186-290."""

    def __init__(self, cin, cout, k, style_dim, demodulate=True, upsample=False):
        super().__init__()
        self.in_channel, self.out_channel, self.kernel_size = cin, cout, k
        self.demodulate, self.upsample = demodulate, upsample
        if upsample:
            self.blur = _Blur(factor=2)
        self.scale = 1 / math.sqrt(cin * k * k)
        self.weight = nn.Parameter(torch.zeros(1, cout, cin, k, k))
        self.modulation = EqualLinearParams(style_dim, cin, bias_init=1)


class _NoiseInjection(nn.Module):
    def __init__(self):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(1))


class StyledConvParams(nn.Module):
    """gpen_model.py:323-363 (isconcat=True: the activation has 2*out bias channels)."""

    def __init__(self, cin, cout, k, style_dim, upsample=False):
        super().__init__()
        self.conv = GPENModulatedConv2dParams(cin, cout, k, style_dim, True, upsample)
        self.noise = _NoiseInjection()
        self.activate = FusedLeakyReLUParams(2 * cout)


class GPENToRGBParams(nn.Module):
    """gpen_model.py:365-384."""

    def __init__(self, cin, style_dim, upsample=True):
        super().__init__()
        if upsample:
            self.upsample = _Upsample()
        self.conv = GPENModulatedConv2dParams(cin, 3, 1, style_dim, demodulate=False)
        self.bias = nn.Parameter(torch.zeros(1, 3, 1, 1))


class _GPENConstantInput(nn.Module):
    def __init__(self, c, size=4):
        super().__init__()
        self.input = nn.Parameter(torch.zeros(1, c, size, size))


class GPENGeneratorParams(nn.Module):
    """gpen_model.py:386-440 (isconcat=True)."""

    def __init__(self, size, style_dim, n_mlp, channel_multiplier=2, lr_mlp=0.01, narrow=1):
        super().__init__()
        self.size, self.n_mlp, self.style_dim = size, n_mlp, style_dim
        layers = [nn.Identity()]                           # PixelNorm
        for _ in range(n_mlp):
            layers.append(EqualLinearParams(style_dim, style_dim, lr_mul=lr_mlp, activation="fused_lrelu"))
        self.style = nn.Sequential(*layers)
        ch = stylegan_channels(channel_multiplier, narrow)
        self.channels = ch
        self.input = _GPENConstantInput(ch[4])
        self.conv1 = StyledConvParams(ch[4], ch[4], 3, style_dim)
        self.to_rgb1 = GPENToRGBParams(ch[4] * 2, style_dim, upsample=False)
        self.log_size = int(math.log(size, 2))
        self.convs = nn.ModuleList()
        self.to_rgbs = nn.ModuleList()
        cin = ch[4]
        for i in range(3, self.log_size + 1):
            cout = ch[2 ** i]
            self.convs.append(StyledConvParams(cin * 2, cout, 3, style_dim, upsample=True))
            self.convs.append(StyledConvParams(cout * 2, cout, 3, style_dim))
            self.to_rgbs.append(GPENToRGBParams(cout * 2, style_dim))
            cin = cout
        self.n_latent = self.log_size * 2 - 2


class ConvLayerParams(nn.Sequential):
    """gpen_model.py:515-562: [Blur] -> EqualConv2d -> FusedLeakyReLU (activate, bias)."""

    def __init__(self, cin, cout, k, downsample=False, bias=True, activate=True):
        layers = []
        if downsample:
            layers.append(_Blur())
        layers.append(EqualConv2dParams(cin, cout, k, stride=2 if downsample else 1,
                                        padding=0 if downsample else k // 2, bias=bias and not activate))
        if activate and bias:
            layers.append(FusedLeakyReLUParams(cout))
        elif activate:
            raise NotImplementedError("ScaledLeakyReLU ConvLayer is not on the FullGenerator path")
        self.downsample, self.activate = downsample, activate
        super().__init__(*layers)


class FullGeneratorParams(nn.Module):
    """gpen_model.py:583-630: encoder ecd0..ecd{log-2} + the StyleGAN2 generator."""

    def __init__(self, size, style_dim, n_mlp, channel_multiplier=2, blur_kernel=(1, 3, 3, 1), lr_mlp=0.01,
                 isconcat=True, narrow=1, device="cpu"):
        super().__init__()
        if not isconcat or tuple(blur_kernel) != (1, 3, 3, 1):
            raise NotImplementedError("FullGenerator: only isconcat=True with the [1,3,3,1] blur is on the path")
        ch = stylegan_channels(channel_multiplier, narrow)
        self.log_size = int(math.log(size, 2))
        self.size, self.style_dim = size, style_dim
        self.generator = GPENGeneratorParams(size, style_dim, n_mlp, channel_multiplier, lr_mlp, narrow)
        self.ecd0 = nn.Sequential(ConvLayerParams(3, ch[size], 1))
        cin = ch[size]
        self.names = [f"ecd{i}" for i in range(self.log_size - 1)]
        for i in range(self.log_size, 2, -1):
            cout = ch[2 ** (i - 1)]
            setattr(self, self.names[self.log_size - i + 1], nn.Sequential(ConvLayerParams(cin, cout, 3, downsample=True)))
            cin = cout
        self.final_linear = nn.Sequential(EqualLinearParams(ch[4] * 16, style_dim, activation="fused_lrelu"))
