"""Parameter layouts of the reference networks.

These classes only *declare* parameters and buffers, under exactly the attribute paths the
reference modules use, so ``state_dict()`` keys, shapes and the spectral-norm
``weight_orig / weight_u / weight_v`` triples match a reference checkpoint one-to-one
(reference loaders: models/__init__.py:12-27, :50-56).  None of them has a forward: the compute
lives in ``s2v_amd.runtime`` (HIP kernels behind the C-ABI library).

Reference layouts mirrored here:
  LNet           models/LNet.py:80-120, base_blocks.py:79-126, :368-457, ffc.py:62-211, transformer.py:58-112
  ENet           models/ENet.py:8-80, base_blocks.py:29-49, :460-554
  DNet           models/DNet.py:13-118, base_blocks.py:127-365
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn.utils import spectral_norm as _torch_spectral_norm


# ----------------------------------------------------------------------------- primitives
def _conv(cin, cout, k, stride=1, padding=0, bias=True, spect=False, padding_mode="zeros", dilation=1):
    c = nn.Conv2d(cin, cout, k, stride, padding, dilation=dilation, bias=bias, padding_mode=padding_mode)
    return _torch_spectral_norm(c) if spect else c


class LayerNorm2dParams(nn.Module):
    """weight/bias [C,1,1] (base_blocks.py:52-69)."""

    def __init__(self, c):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c, 1, 1))
        self.bias = nn.Parameter(torch.zeros(c, 1, 1))


class ConvNormAct(nn.Module):
    """FirstBlock2d / DownBlock2d / UpBlock2d / Jump: model = [conv, LayerNorm2d, act(, pool)]."""

    def __init__(self, cin, cout, k, spect, pool=False):
        super().__init__()
        layers = [_conv(cin, cout, k, 1, k // 2, spect=spect), LayerNorm2dParams(cout), nn.LeakyReLU(0.1)]
        if pool:
            layers.append(nn.AvgPool2d(2))
        self.model = nn.Sequential(*layers)


class FinalConv(nn.Module):
    """FinalBlock2d (base_blocks.py:444-457): model = [conv7x7, sigmoid|tanh]."""

    def __init__(self, cin, cout, spect, act):
        super().__init__()
        self.act = act
        self.model = nn.Sequential(_conv(cin, cout, 7, 1, 3, spect=spect),
                                   nn.Sigmoid() if act == "sigmoid" else nn.Tanh())


class ADAINParams(nn.Module):
    """ADAIN (base_blocks.py:127-157): mlp_shared.0, mlp_gamma, mlp_beta."""

    def __init__(self, norm_nc, feature_nc, nhidden=128):
        super().__init__()
        self.norm_nc, self.feature_nc, self.nhidden = norm_nc, feature_nc, nhidden
        self.mlp_shared = nn.Sequential(nn.Linear(feature_nc, nhidden), nn.ReLU())
        self.mlp_gamma = nn.Linear(nhidden, norm_nc)
        self.mlp_beta = nn.Linear(nhidden, norm_nc)


class AudioConvParams(nn.Module):
    """models/base_blocks.py:12-26 Conv2d: conv_block = [Conv2d, BatchNorm2d], optional residual."""

    def __init__(self, cin, cout, k, stride, padding, residual=False):
        super().__init__()
        self.cfg = dict(k=k, stride=stride if isinstance(stride, tuple) else (stride, stride),
                        padding=padding, residual=residual)
        self.conv_block = nn.Sequential(nn.Conv2d(cin, cout, k, stride, padding), nn.BatchNorm2d(cout))


# ----------------------------------------------------------------------------- FFC
class FourierUnitParams(nn.Module):
    """ffc.py:62-87 (spectral_pos_encoding / use_se off on this path)."""

    def __init__(self, c):
        super().__init__()
        self.conv_layer = nn.Conv2d(2 * c, 2 * c, 1, bias=False)
        self.bn = nn.BatchNorm2d(2 * c)


class SpectralTransformParams(nn.Module):
    """ffc.py:129-153 with stride 1 and enable_lfu=False (base_blocks.py:375-377)."""

    def __init__(self, cin, cout):
        super().__init__()
        self.downsample = nn.Identity()
        self.conv1 = nn.Sequential(nn.Conv2d(cin, cout // 2, 1, bias=False), nn.BatchNorm2d(cout // 2), nn.ReLU())
        self.fu = FourierUnitParams(cout // 2)
        self.conv2 = nn.Conv2d(cout // 2, cout, 1, bias=False)


class FFCParams(nn.Module):
    """ffc.py:176-211, kernel 3, ratio 0.75/0.75, reflect padding."""

    def __init__(self, c, ratio=0.75):
        super().__init__()
        cg = int(c * ratio)
        cl = c - cg
        self.global_in_num = cg
        self.in_cl, self.in_cg = cl, cg
        kw = dict(bias=False, padding_mode="reflect")
        self.convl2l = nn.Conv2d(cl, cl, 3, 1, 1, **kw)
        self.convl2g = nn.Conv2d(cl, cg, 3, 1, 1, **kw)
        self.convg2l = nn.Conv2d(cg, cl, 3, 1, 1, **kw)
        self.convg2g = SpectralTransformParams(cg, cg)
        self.gate = nn.Identity()


class FineADAINLamaParams(nn.Module):
    """base_blocks.py:368-386."""

    def __init__(self, c, feature_nc):
        super().__init__()
        self.ffc = FFCParams(c)
        self.bn_l = ADAINParams(c - self.ffc.global_in_num, feature_nc)
        self.bn_g = ADAINParams(self.ffc.global_in_num, feature_nc)


class FFCResnetBlockParams(nn.Module):
    """base_blocks.py:389-411 (inline=True)."""

    def __init__(self, c, feature_nc):
        super().__init__()
        self.conv1 = FineADAINLamaParams(c, feature_nc)
        self.conv2 = FineADAINLamaParams(c, feature_nc)


class ResBlocksParams(nn.Module):
    """FFCADAINResBlocks / FineADAINResBlocks: res0..res{n-1}."""

    def __init__(self, n, make):
        super().__init__()
        self.num_block = n
        for i in range(n):
            setattr(self, f"res{i}", make())


# ----------------------------------------------------------------------------- transformer
class _LN(nn.LayerNorm):
    pass


class AttentionParams(nn.Module):
    """transformer.py:36-68 (q, k from x; v from y)."""

    def __init__(self, dim, heads, dim_head):
        super().__init__()
        inner = heads * dim_head
        self.heads, self.dim_head = heads, dim_head
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_k = nn.Linear(dim, inner, bias=False)
        self.to_v = nn.Linear(dim, inner, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(0.0))


class DualPreNormParams(nn.Module):
    def __init__(self, dim, fn):
        super().__init__()
        self.normx = nn.LayerNorm(dim)
        self.normy = nn.LayerNorm(dim)
        self.fn = fn


class FeedForwardParams(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(dim, hidden), nn.Identity(), nn.Dropout(0.0),
                                 nn.Linear(hidden, dim), nn.Dropout(0.0))


class PreNormParams(nn.Module):
    def __init__(self, dim, fn):
        super().__init__()
        self.norm = nn.LayerNorm(dim)
        self.fn = fn


class TransformerParams(nn.Module):
    """transformer.py:89-112: depth x [DualPreNorm(Attention), PreNorm(FeedForward)]."""

    def __init__(self, dim, depth, heads, dim_head, mlp_dim):
        super().__init__()
        self.layers = nn.ModuleList([
            nn.ModuleList([DualPreNormParams(dim, AttentionParams(dim, heads, dim_head)),
                           PreNormParams(dim, FeedForwardParams(dim, mlp_dim))])
            for _ in range(depth)])


# ----------------------------------------------------------------------------- LNet
class VisualEncoderParams(nn.Module):
    """LNet.py:10-43."""

    def __init__(self, image_nc=3, ngf=64, img_f=512, layers=3, spect=True):
        super().__init__()
        self.layers = layers
        self.first_inp = ConvNormAct(image_nc, ngf, 7, spect)
        self.first_ref = ConvNormAct(image_nc, ngf, 7, spect)
        for i in range(layers):
            cin, cout = min(ngf * 2 ** i, img_f), min(ngf * 2 ** (i + 1), img_f)
            setattr(self, f"ca{i}", nn.Identity() if i < 2 else
                    TransformerParams(2 ** (i + 1) * ngf, 2, 4, ngf, ngf * 4))
            setattr(self, f"ref_down{i}", ConvNormAct(cin, cout, 3, spect, pool=True))
            setattr(self, f"inp_down{i}", ConvNormAct(cin, cout, 3, spect, pool=True))


class LNetDecoderParams(nn.Module):
    """LNet.py:46-77."""

    def __init__(self, image_nc=3, feature_nc=512, ngf=64, img_f=512, layers=3, num_block=9, spect=True):
        super().__init__()
        self.layers = layers
        for i in reversed(range(layers)):
            cin = ngf * 2 ** (i + 1) * 2 if i == layers - 1 else min(ngf * 2 ** (i + 1), img_f)
            cout = min(ngf * 2 ** i, img_f)
            setattr(self, f"up{i}", ConvNormAct(cin, cout, 3, spect))
            setattr(self, f"res{i}", ResBlocksParams(num_block, lambda c=cin: FFCResnetBlockParams(c, feature_nc)))
            setattr(self, f"jump{i}", ConvNormAct(cout, cout, 3, spect))
        self.final = FinalConv(cout, image_nc, spect, "sigmoid")


_AUDIO_LAYERS = [  # LNet.py:102-120: (cin, cout, k, stride, padding, residual)
    (1, 32, 3, 1, 1, False), (32, 32, 3, 1, 1, True), (32, 32, 3, 1, 1, True),
    (32, 64, 3, (3, 1), 1, False), (64, 64, 3, 1, 1, True), (64, 64, 3, 1, 1, True),
    (64, 128, 3, 3, 1, False), (128, 128, 3, 1, 1, True), (128, 128, 3, 1, 1, True),
    (128, 256, 3, (3, 2), 1, False), (256, 256, 3, 1, 1, True),
    (256, 512, 3, 1, 0, False), (512, 512, 1, 1, 0, False),
]


class LNetParams(nn.Module):
    """LNet (models/LNet.py:80-120) parameter layout."""

    def __init__(self, image_nc=3, descriptor_nc=512, layer=3, base_nc=64, max_nc=512,
                 num_res_blocks=9, use_spect=True):
        super().__init__()
        self.descriptor_nc = descriptor_nc
        self.encoder = VisualEncoderParams(image_nc, base_nc, max_nc, layer, use_spect)
        self.decoder = LNetDecoderParams(image_nc, descriptor_nc, base_nc, max_nc, layer, num_res_blocks, use_spect)
        layers = list(_AUDIO_LAYERS)
        layers[-1] = (512, descriptor_nc, 1, 1, 0, False)
        self.audio_encoder = nn.Sequential(*[AudioConvParams(*cfg) for cfg in layers])


# ----------------------------------------------------------------------------- ENet
class ResBlockParams(nn.Module):
    """base_blocks.py:29-49 (mode='down')."""

    def __init__(self, cin, cout):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cin, 3, 1, 1)
        self.conv2 = nn.Conv2d(cin, cout, 3, 1, 1)
        self.skip = nn.Conv2d(cin, cout, 1, bias=False)


class ModulatedConv2dParams(nn.Module):
    """base_blocks.py:460-508."""

    def __init__(self, cin, cout, k, num_style_feat, demodulate=True, sample_mode=None, eps=1e-8):
        super().__init__()
        self.in_channels, self.out_channels, self.kernel_size = cin, cout, k
        self.demodulate, self.sample_mode, self.eps = demodulate, sample_mode, eps
        self.modulation = nn.Linear(num_style_feat, cin, bias=True)
        self.weight = nn.Parameter(torch.zeros(1, cout, cin, k, k))


class StyleConvParams(nn.Module):
    """base_blocks.py:515-536: weight = noise strength [1], bias [1,C,1,1]."""

    def __init__(self, cin, cout, k, num_style_feat, demodulate=True, sample_mode=None):
        super().__init__()
        self.modulated_conv = ModulatedConv2dParams(cin, cout, k, num_style_feat, demodulate, sample_mode)
        self.weight = nn.Parameter(torch.zeros(1))
        self.bias = nn.Parameter(torch.zeros(1, cout, 1, 1))


class ToRGBParams(nn.Module):
    """base_blocks.py:539-554."""

    def __init__(self, cin, num_style_feat, upsample=True):
        super().__init__()
        self.upsample = upsample
        self.modulated_conv = ModulatedConv2dParams(cin, 3, 1, num_style_feat, demodulate=False)
        self.bias = nn.Parameter(torch.zeros(1, 3, 1, 1))


ENET_CHANNELS = {"4": 512, "8": 512, "16": 512, "32": 512, "64": 512, "128": 256, "256": 128,
                 "512": 64, "1024": 32}


class ENetParams(nn.Module):
    """ENet (models/ENet.py:8-80) parameter layout; ``low_res`` holds the LNet."""

    def __init__(self, num_style_feat=512, lnet=None, concat=False):
        super().__init__()
        if concat:
            raise NotImplementedError("ENet(concat=True) is not on the inference path (ENet.py:134)")
        self.low_res = lnet if lnet is not None else LNetParams()
        for p in self.low_res.parameters():
            p.requires_grad = False
        ch = ENET_CHANNELS
        self.log_size = 8
        self.num_style_feat = num_style_feat
        self.conv_body_first = nn.Conv2d(3, ch["128"], 1)
        self.conv_body_down = nn.ModuleList()
        cin = ch["128"]
        for i in range(8, 2, -1):
            cout = ch[f"{2 ** (i - 1)}"]
            self.conv_body_down.append(ResBlockParams(cin, cout))
            cin = cout
        self.final_linear = nn.Linear(ch["4"] * 4 * 4, num_style_feat)
        self.final_conv = nn.Conv2d(cin, ch["4"], 3, 1, 1)
        self.style_convs = nn.ModuleList()
        self.to_rgbs = nn.ModuleList()
        self.noises = nn.Module()
        self.concat = concat
        cin = 3
        for i in range(7, 9):
            cout = ch[f"{2 ** i}"]
            self.style_convs.append(StyleConvParams(cin, cout, 3, num_style_feat, True, "upsample"))
            self.style_convs.append(StyleConvParams(cout, cout, 3, num_style_feat, True, None))
            self.to_rgbs.append(ToRGBParams(cout, num_style_feat, upsample=True))
            cin = cout


# ----------------------------------------------------------------------------- DNet
class MappingNetParams(nn.Module):
    """DNet.py:30-54."""

    def __init__(self, coeff_nc=73, descriptor_nc=256, layer=3):
        super().__init__()
        self.layer = layer
        self.first = nn.Sequential(nn.Conv1d(coeff_nc, descriptor_nc, 7, padding=0, bias=True))
        for i in range(layer):
            setattr(self, f"encoder{i}", nn.Sequential(
                nn.LeakyReLU(0.1), nn.Conv1d(descriptor_nc, descriptor_nc, 3, padding=0, dilation=3)))
        self.pooling = nn.AdaptiveAvgPool1d(1)
        self.output_nc = descriptor_nc


class ADAINEncoderBlockParams(nn.Module):
    """base_blocks.py:195-212."""

    def __init__(self, cin, cout, feature_nc):
        super().__init__()
        self.conv_0 = nn.Conv2d(cin, cout, 4, 2, 1)
        self.conv_1 = nn.Conv2d(cout, cout, 3, 1, 1)
        self.norm_0 = ADAINParams(cin, feature_nc)
        self.norm_1 = ADAINParams(cout, feature_nc)


class ADAINDecoderBlockParams(nn.Module):
    """base_blocks.py:215-252 (use_transpose=True)."""

    def __init__(self, cin, cout, hidden, feature_nc):
        super().__init__()
        hidden = min(cin, cout) if hidden is None else hidden
        self.conv_0 = nn.Conv2d(cin, hidden, 3, 1, 1)
        self.conv_1 = nn.ConvTranspose2d(hidden, cout, 3, 2, 1, output_padding=1)
        self.conv_s = nn.ConvTranspose2d(cin, cout, 3, 2, 1, output_padding=1)
        self.norm_0 = ADAINParams(cin, feature_nc)
        self.norm_1 = ADAINParams(hidden, feature_nc)
        self.norm_s = ADAINParams(cin, feature_nc)


class ADAINEncoderParams(nn.Module):
    def __init__(self, image_nc, pose_nc, ngf, img_f, layers):
        super().__init__()
        self.layers = layers
        self.input_layer = nn.Conv2d(image_nc, ngf, 7, 1, 3)
        for i in range(layers):
            cin, cout = min(ngf * 2 ** i, img_f), min(ngf * 2 ** (i + 1), img_f)
            setattr(self, f"encoder{i}", ADAINEncoderBlockParams(cin, cout, pose_nc))


class ADAINDecoderParams(nn.Module):
    def __init__(self, pose_nc, ngf, img_f, encoder_layers, decoder_layers):
        super().__init__()
        self.encoder_layers, self.decoder_layers = encoder_layers, decoder_layers
        for i in reversed(range(encoder_layers - decoder_layers, encoder_layers)):
            cin = min(ngf * 2 ** (i + 1), img_f)
            cin = cin * 2 if i != encoder_layers - 1 else cin
            cout = min(ngf * 2 ** i, img_f)
            setattr(self, f"decoder{i}", ADAINDecoderBlockParams(cin, cout, cout, pose_nc))
        self.output_nc = cout * 2


class ADAINHourglassParams(nn.Module):
    def __init__(self, image_nc, pose_nc, ngf, img_f, encoder_layers, decoder_layers):
        super().__init__()
        self.encoder = ADAINEncoderParams(image_nc, pose_nc, ngf, img_f, encoder_layers)
        self.decoder = ADAINDecoderParams(pose_nc, ngf, img_f, encoder_layers, decoder_layers)
        self.output_nc = self.decoder.output_nc


class WarpingNetParams(nn.Module):
    """DNet.py:56-90."""

    def __init__(self, image_nc=3, descriptor_nc=256, base_nc=32, max_nc=256, encoder_layer=5, decoder_layer=3):
        super().__init__()
        self.descriptor_nc = descriptor_nc
        self.hourglass = ADAINHourglassParams(image_nc, descriptor_nc, base_nc, max_nc, encoder_layer, decoder_layer)
        c = self.hourglass.output_nc
        self.flow_out = nn.Sequential(LayerNorm2dParams(c), nn.LeakyReLU(0.1), nn.Conv2d(c, 2, 7, 1, 3))
        self.pool = nn.AdaptiveAvgPool2d(1)


class FineADAINResBlock2dParams(nn.Module):
    """base_blocks.py:160-177 (conv1/norm1 are declared but dead in the forward)."""

    def __init__(self, c, feature_nc):
        super().__init__()
        self.conv1 = nn.Conv2d(c, c, 3, 1, 1)
        self.conv2 = nn.Conv2d(c, c, 3, 1, 1)
        self.norm1 = ADAINParams(c, feature_nc)
        self.norm2 = ADAINParams(c, feature_nc)


class FineEncoderParams(nn.Module):
    """base_blocks.py:255-275."""

    def __init__(self, image_nc, ngf, img_f, layers):
        super().__init__()
        self.layers = layers
        self.first = ConvNormAct(image_nc, ngf, 7, False)
        for i in range(layers):
            cin, cout = min(ngf * 2 ** i, img_f), min(ngf * 2 ** (i + 1), img_f)
            setattr(self, f"down{i}", ConvNormAct(cin, cout, 3, False, pool=True))


class FineDecoderParams(nn.Module):
    """base_blocks.py:278-305."""

    def __init__(self, image_nc, feature_nc, ngf, img_f, layers, num_block):
        super().__init__()
        self.layers = layers
        for i in reversed(range(layers)):
            cin, cout = min(ngf * 2 ** (i + 1), img_f), min(ngf * 2 ** i, img_f)
            setattr(self, f"up{i}", ConvNormAct(cin, cout, 3, False))
            setattr(self, f"res{i}", ResBlocksParams(num_block, lambda c=cin: FineADAINResBlock2dParams(c, feature_nc)))
            setattr(self, f"jump{i}", ConvNormAct(cout, cout, 3, False))
        self.final = FinalConv(cout, image_nc, False, "tanh")


class EditingNetParams(nn.Module):
    """DNet.py:93-118."""

    def __init__(self, image_nc=3, descriptor_nc=256, layer=3, base_nc=64, max_nc=256, num_res_blocks=2):
        super().__init__()
        self.descriptor_nc = descriptor_nc
        self.encoder = FineEncoderParams(image_nc * 2, base_nc, max_nc, layer)
        self.decoder = FineDecoderParams(image_nc, descriptor_nc, base_nc, max_nc, layer, num_res_blocks)


class DNetParams(nn.Module):
    """DNet (models/DNet.py:13-28) parameter layout."""

    def __init__(self):
        super().__init__()
        self.mapping_net = MappingNetParams()
        self.warpping_net = WarpingNetParams()
        self.editing_net = EditingNetParams()
