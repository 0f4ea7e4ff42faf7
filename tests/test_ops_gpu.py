"""Per-kernel parity of libs2v (called through the C ABI) against fp64 CPU references.

fp32 kernels vs fp64 references: tolerances are stated per test.  The implicit-GEMM convolutions
run in both arithmetic modes (``prec`` fixture):
  * f32    (v_mfma_f32_32x32x2_f32): 2e-6 * sum|a*b| (k-ordered fp32 fma chains, < 1.5e-7*K
           relative to that sum for K <= 10^4, cdna_hip_programming.md §3 'FP32-input MFMA');
  * bf16x3 (split-fp32 on v_mfma_f32_32x32x16_bf16): 5e-5 * sum|a*b| — worst case per product:
           each operand's hi + lo is within 2^-16 of it and the dropped |al*bl| <= 2^-16 |a*b|,
           so 3 * 2^-16 = 4.6e-5 relative, plus the fp32 sums;
  * f16x3  (the same split on v_mfma_f32_32x32x16_f16): 3e-6 * sum|a*b| — 3 * 2^-22 = 7.2e-7 per
           product in the f16 normal range (weights pre-scaled into it), plus the fp32 sums.
"""
import ctypes
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import s2v_import  # noqa: F401

pytestmark = pytest.mark.gpu

from s2v_amd import ops  # noqa: E402  (importable without a device; launches need one)
from s2v_amd.ops import NHWC, ConvW  # noqa: E402

DEV = "cuda"


REL = {"f32": 2e-6, "bf16x3": 5e-5, "f16x3": 3e-6}


@pytest.fixture(scope="module")
def ctx():
    return ops.Ctx(DEV)




def nhwc(t):
    return NHWC(t.permute(0, 2, 3, 1).contiguous().to(DEV))


def to_nchw(v: NHWC):
    return v.t[..., v.coff: v.coff + v.c].permute(0, 3, 1, 2).double().cpu()


def rnd(*shape, seed=0, lo=-1.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return lo + (hi - lo) * torch.rand(*shape, generator=g, dtype=torch.float64)


def act_ref(v, act, alpha):
    if act == ops.ACT_RELU:
        return F.relu(v)
    if act == ops.ACT_LRELU:
        return F.leaky_relu(v, alpha)
    if act == ops.ACT_SIGMOID:
        return torch.sigmoid(v)
    if act == ops.ACT_TANH:
        return torch.tanh(v)
    if act == ops.ACT_GELU_TANH:
        return 0.5 * v * (1 + torch.tanh(math.sqrt(2 / math.pi) * (v + 0.044715 * v ** 3)))
    return v


def conv_bound(x, w, stride, padding, dilation, transposed=False, op=0):
    f = F.conv_transpose2d if transposed else F.conv2d
    kw = dict(stride=stride, padding=padding, dilation=dilation)
    if transposed:
        kw["output_padding"] = op
    return f(x.abs(), w.abs(), **kw)


CONV_CASES = [
    # (n, cin, h, w, cout, k, stride, pad, dil, mode, pad_mode, tile, splits)
    (2, 64, 17, 19, 96, 3, 1, 1, 1, "direct", "zero", 0, 0),
    (2, 64, 16, 16, 256, 3, 1, 1, 1, "direct", "zero", 1, 0),     # 256-wide N tile needs cout > 128
    (2, 64, 16, 16, 128, 3, 1, 1, 1, "direct", "zero", 2, 3),
    (1, 32, 20, 12, 64, 3, 2, 1, 1, "direct", "zero", 3, 0),
    (2, 32, 12, 12, 64, 3, 1, 1, 1, "direct", "zero", 4, 2),
    # 64x64 tile (force_tile 5) with cout 32 < BN: the N tail of the B loads and the epilogue
    (2, 32, 12, 12, 32, 3, 1, 1, 1, "direct", "zero", 5, 0),
    (2, 64, 17, 15, 32, 3, 1, 1, 1, "direct", "reflect", 5, 2),
    (2, 96, 10, 10, 200, 3, 1, 1, 1, "direct", "reflect", 5, 0),
    (2, 48, 12, 12, 40, 3, 1, 1, 1, "direct", "reflect", 6, 4),
    (1, 3, 24, 24, 64, 7, 1, 3, 1, "direct", "zero", 0, 0),
    (2, 6, 20, 20, 33, 4, 2, 1, 1, "direct", "zero", 0, 0),
    (2, 73, 1, 26, 40, (1, 7), 1, 0, 1, "direct", "zero", 0, 0),
    (2, 40, 1, 20, 40, (1, 3), 1, 0, (1, 3), "direct", "zero", 0, 0),
    (2, 32, 8, 8, 48, 3, 1, 1, 1, "up2", "zero", 0, 0),
    (2, 64, 6, 7, 32, 3, 2, 1, 1, "transposed", "zero", 0, 0),
    (2, 64, 9, 9, 3, 7, 1, 3, 1, "direct", "zero", 0, 0),     # direct small-N kernel
    # halo-tiled small-Cout kernel (8 x 128 output tiles): ragged tiles in both directions, reflect
    # halos, 3 / 5 / 7 filters, 1..4 outputs (DNet's 7x7 64 -> 3 head at 256^2 is the model case);
    # rows with w >= 96 run it with the planner's block-count floor off (halo_everywhere)
    (2, 64, 37, 150, 3, 7, 1, 3, 1, "direct", "zero", 0, 0),
    (1, 64, 20, 130, 3, 7, 1, 3, 1, "direct", "reflect", 0, 0),
    (2, 32, 19, 100, 4, 3, 1, 1, 1, "direct", "reflect", 0, 0),
    (2, 16, 16, 120, 1, 5, 1, 2, 1, "direct", "zero", 0, 0),
    (2, 32, 19, 17, 4, 3, 1, 1, 1, "direct", "reflect", 0, 0),      # narrow: channel-parallel kernel
    (2, 16, 16, 16, 1, 5, 1, 2, 1, "direct", "zero", 0, 0),
    (1, 8, 9, 260, 2, 7, 1, 2, 1, "direct", "zero", 0, 0),
    (3, 1, 20, 16, 32, 3, (3, 1), 1, 1, "direct", "zero", 0, 0),
    (2, 128, 3, 3, 256, 3, (3, 2), 1, 1, "direct", "zero", 0, 0),
    # small-K direct kernel (K = kh*kw*cin <= 64, cin % 4 == 0): image-input / 4-channel layers
    (2, 4, 17, 19, 64, 3, 1, 1, 1, "direct", "zero", 0, 0),
    (2, 4, 16, 16, 256, 1, 1, 0, 1, "direct", "zero", 0, 0),
    (1, 4, 9, 9, 512, 1, 1, 0, 1, "direct", "zero", 0, 0),
    (2, 4, 33, 35, 256, 1, 1, 0, 1, "direct", "zero", 0, 0),        # 1x1 load groups with a ragged tail
    (2, 4, 10, 12, 32, 3, 1, 1, 1, "direct", "reflect", 0, 0),
    (2, 4, 8, 8, 64, 3, 1, 1, 1, "up2", "zero", 0, 0),
    (2, 4, 14, 14, 128, 3, 2, 1, 1, "direct", "zero", 0, 0),
    # nearest-x2 input with reflect padding (ParseNet 'up' ConvLayers, blocks.py:92-96): per-row
    # index path (cin % 32), float4 gather, small-K and small-Cout kernels
    (2, 64, 9, 7, 64, 3, 1, 1, 1, "up2", "reflect", 0, 0),
    (2, 36, 5, 6, 40, 3, 1, 1, 1, "up2", "reflect", 0, 0),
    (2, 4, 8, 8, 64, 3, 1, 1, 1, "up2", "reflect", 0, 0),
    (2, 64, 6, 6, 3, 3, 1, 1, 1, "up2", "reflect", 0, 0),
    (2, 64, 12, 12, 48, 3, 1, 1, 1, "up2", "zero", 4, 2),
    # bf16x3 256x128 8-wave tile (force_tile 7; the f32 table has 6 tiles)
    (2, 64, 18, 16, 128, 3, 1, 1, 1, "direct", "zero", 7, 0),
    (2, 96, 10, 11, 72, 3, 1, 1, 1, "up2", "reflect", 7, 2),
    # bf16x3 256x64 8-wave tile (force_tile 8: large-M, 64-channel layers)
    (2, 64, 20, 18, 64, 3, 1, 1, 1, "direct", "reflect", 8, 0),
    (1, 32, 17, 23, 40, 3, 2, 1, 1, "direct", "zero", 8, 3),
    # narrow-N tiles with 64-row waves (force_tile 10 / 11 / 12: 512x64 8-wave, 256x64 and 256x32 4-wave):
    # ragged M / N tails, split-K, reflect padding (per-row gather), up2
    (2, 64, 23, 29, 64, 3, 1, 1, 1, "direct", "zero", 10, 0),
    (1, 96, 19, 21, 40, 3, 1, 1, 1, "direct", "reflect", 10, 3),
    (2, 64, 17, 15, 64, 3, 1, 1, 1, "direct", "zero", 11, 2),
    (2, 32, 9, 10, 48, 3, 1, 1, 1, "up2", "zero", 11, 0),
    (2, 64, 20, 18, 32, 3, 1, 1, 1, "direct", "zero", 12, 0),
    (1, 128, 13, 17, 24, 3, 2, 1, 1, "direct", "zero", 12, 4),
    # conv_x3_nar (force_tile 16: register-direct A fragments, 256x64; 17: B fragments too): ragged M,
    # N < 64, several N tiles, stride 2, split-K, 1x1
    (2, 64, 23, 29, 64, 3, 1, 1, 1, "direct", "zero", 16, 0),
    (2, 64, 23, 29, 64, 3, 1, 1, 1, "direct", "zero", 17, 2),
    (2, 32, 17, 15, 130, 3, 2, 1, 1, "direct", "zero", 17, 0),
    (1, 96, 19, 21, 40, 3, 1, 1, 1, "direct", "zero", 16, 3),
    (2, 32, 17, 15, 130, 3, 2, 1, 1, "direct", "zero", 16, 0),
    (2, 64, 11, 13, 96, 1, 1, 0, 1, "direct", "zero", 16, 2),
    # conv_x3_halo (force_tile 18: 4 x 64 patches x 64 channels; 20: x 128 channels): every epilogue
    # variant of the test (incl. the output slice of a wider tensor), ragged patches, split-K
    (2, 64, 12, 64, 64, 3, 1, 1, 1, "direct", "zero", 18, 0),
    (1, 96, 9, 70, 100, 3, 1, 1, 1, "direct", "zero", 20, 2),
    (2, 32, 5, 130, 40, 3, 1, 1, 1, "direct", "zero", 18, 0),
    # 1x1 Cout <= 4 heads (conv_small_cpar, LDS weights; 2 / 4 / 8 lanes per pixel, 4 / 8 float4s
    # per lane)
    (2, 64, 17, 19, 3, 1, 1, 0, 1, "direct", "zero", 0, 0),
    (1, 128, 9, 33, 2, 1, 1, 0, 1, "direct", "zero", 0, 0),
    (2, 32, 7, 11, 4, 1, 1, 0, 1, "direct", "zero", 0, 0),
    (1, 256, 5, 9, 1, 1, 1, 0, 1, "direct", "zero", 0, 0),
]


@pytest.mark.parametrize("shape", [(4, 64, 32, 48, 64, 3, 1), (2, 128, 32, 40, 48, 3, 1), (2, 64, 64, 64, 64, 3, 2),
                                   (3, 32, 16, 96, 64, 1, 1)])
def test_conv_nar_bit_identical_to_lds_tile(ctx, prec, shape):
    """conv_x3_nar (A fragments straight to registers; force_tile 17: B too) against the LDS-staged
    256x64 4-wave tile (force_tile 11): same K order, same split, same MFMA order per slice -> bit-identical outputs, with
    the StyleGAN2 input modulation (in_scale, per image: tiles inside one image and tiles straddling two),
    a pre-activation, the demodulation / noise / residual epilogue."""
    if prec == "f32":
        pytest.skip("split precisions only")
    n, cin, h, w, cout, k, st = shape
    wt = rnd(cout, cin, k, k, seed=41) / math.sqrt(cin * k * k)
    cw = ConvW(wt.float(), rnd(cout, seed=42).float(), DEV, stride=st, padding=k // 2)
    x = nhwc(rnd(n, cin, h, w, seed=43).float())
    oh, ow = (h + 2 * (k // 2) - k) // st + 1, (w + 2 * (k // 2) - k) // st + 1
    s = rnd(n, cin, seed=44, lo=0.5, hi=1.5).float().to(DEV)
    d = rnd(n, cout, seed=45, lo=0.5, hi=1.5).float().to(DEV)
    noise = rnd(n, oh * ow, seed=46).float().to(DEV)
    res = nhwc(rnd(n, cout, oh, ow, seed=47).float())
    for kw in (dict(), dict(in_scale=s, nc_scale=d, pix_add=noise, pix_w=0.3, act=ops.ACT_LRELU, alpha=0.2),
               dict(pre_act=ops.ACT_LRELU, pre_alpha=0.2, res=res, act=ops.ACT_TANH), dict(force_splits=2)):
        outs = []
        for tile in (11, 16, 17):
            y = NHWC.empty(n, oh, ow, cout, DEV)
            ops.conv2d(ctx, x, cw, y, force_tile=tile, **kw)
            outs.append(y.t.clone())
        torch.cuda.synchronize()
        for o in outs[1:]:
            assert torch.equal(outs[0], o), f"{kw.keys()}: max diff {(outs[0] - o).abs().max():.3e}"
    xs = nhwc(rnd(n, cin, 10, 10, seed=48).float())
    with pytest.raises(Exception, match="conv_x3_nar"):
        ops.conv2d(ctx, xs, cw, NHWC.empty(n, (10 + 2 * (k // 2) - k) // st + 1, (10 + 2 * (k // 2) - k) // st + 1,
                                           cout, DEV), force_tile=16, in_scale=s)


@pytest.mark.parametrize("shape", [(2, 64, 8, 128, 64), (1, 96, 4, 64, 40), (2, 32, 12, 64, 130), (4, 128, 16, 64, 64),
                                   (2, 64, 10, 100, 64), (1, 32, 7, 70, 96)])
def test_conv_halo_bit_identical_to_lds_tile(ctx, prec, shape):
    """conv_x3_halo (force_tile 18 / 19 / 20: 4 x 64 / 8 x 64 output patches, 20 with 128 output channels
    per block; the input halo split once per channel slice)
    against the LDS-staged 256x64 tile (force_tile 11): same K order (taps fastest within a channel
    slice), same MFMA order -> bit-identical, with modulation, pre-activation, demod / noise / residual
    epilogues; ragged images (partly empty last patches); halo split-K (whole channel slices) against
    the unsplit launch at the split bound; a strided conv is refused when forced."""
    if prec == "f32":
        pytest.skip("split precisions only")
    n, cin, h, w, cout = shape
    wt = rnd(cout, cin, 3, 3, seed=51) / math.sqrt(cin * 9)
    cw = ConvW(wt.float(), rnd(cout, seed=52).float(), DEV, padding=1)
    x = nhwc(rnd(n, cin, h, w, seed=53).float())
    s = rnd(n, cin, seed=54, lo=0.5, hi=1.5).float().to(DEV)
    d = rnd(n, cout, seed=55, lo=0.5, hi=1.5).float().to(DEV)
    noise = rnd(n, h * w, seed=56).float().to(DEV)
    res = nhwc(rnd(n, cout, h, w, seed=57).float())
    for kw in (dict(), dict(in_scale=s, nc_scale=d, pix_add=noise, pix_w=0.3, act=ops.ACT_LRELU, alpha=0.2),
               dict(pre_act=ops.ACT_LRELU, pre_alpha=0.2, res=res, act=ops.ACT_TANH)):
        outs = []
        for tile in (11, 18, 20) + ((19,) if h % 8 == 0 else ()):
            y = NHWC.empty(n, h, w, cout, DEV)
            ops.conv2d(ctx, x, cw, y, force_tile=tile, **kw)
            outs.append(y.t.clone())
        torch.cuda.synchronize()
        for o in outs[1:]:
            assert torch.equal(outs[0], o), f"{kw.keys()}: max diff {(outs[0] - o).abs().max():.3e}"
    if cin >= 64:
        ysp = NHWC.empty(n, h, w, cout, DEV)
        ops.conv2d(ctx, x, cw, ysp, force_tile=18, force_splits=2)
        y1 = NHWC.empty(n, h, w, cout, DEV)
        ops.conv2d(ctx, x, cw, y1, force_tile=18)
        assert (ysp.t - y1.t).abs().max() <= 1e-5 * (y1.t.abs().max() + 1)
    cw2 = ConvW(wt.float(), None, DEV, stride=2, padding=1)
    with pytest.raises(Exception, match="conv_x3_halo"):
        ops.conv2d(ctx, nhwc(rnd(n, cin, 8, 64, seed=58).float()), cw2, NHWC.empty(n, 4, 32, cout, DEV), force_tile=18)


@pytest.fixture
def halo_everywhere(ctx):
    """The halo-tiled small-Cout kernel for every qualifying shape (its block-count floor off), so
    the small test images exercise it."""
    prev = ops.tune(ctx, ops.TUNE_HALO_MIN_BLOCKS, 0)
    yield
    ops.tune(ctx, ops.TUNE_HALO_MIN_BLOCKS, prev)


@pytest.mark.parametrize("case", CONV_CASES, ids=[str(i) for i in range(len(CONV_CASES))])
def test_conv2d(ctx, prec, case, request):
    n, cin, h, w, cout, k, stride, pad, dil, mode, pad_mode, tile, splits = case
    if cout <= 4 and w >= 96:
        request.getfixturevalue("halo_everywhere")
    if tile > 6 and prec == "f32":
        pytest.skip("tiles 7-8 exist in the bf16x3 table only")
    kh, kw = (k, k) if isinstance(k, int) else k
    transposed = mode == "transposed"
    wshape = (cin, cout, kh, kw) if transposed else (cout, cin, kh, kw)
    wt = rnd(*wshape, seed=1) / math.sqrt(cin * kh * kw)
    bias = rnd(cout, seed=2)
    x = rnd(n, cin, h, w, seed=3)
    st = stride if isinstance(stride, tuple) else (stride, stride)
    dl = dil if isinstance(dil, tuple) else (dil, dil)
    cw = ConvW(wt.float(), bias.float(), DEV, stride=st, padding=pad, dilation=dl, transposed=transposed,
               output_padding=1 if transposed else 0,
               pad_mode=ops.PAD_REFLECT if pad_mode == "reflect" else ops.PAD_ZERO,
               in_mode=ops.IN_NEAREST_UP2 if mode == "up2" else ops.IN_DIRECT)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if mode == "up2" else x
    if transposed:
        ref = F.conv_transpose2d(x, wt, bias, st, pad, output_padding=1, dilation=dl)
        bound = conv_bound(x, wt, st, pad, dl, True, 1)
    else:
        xp = F.pad(xin, (pad,) * 4, mode="reflect") if pad_mode == "reflect" else xin
        p = 0 if pad_mode == "reflect" else pad
        ref = F.conv2d(xp, wt, bias, st, p, dl)
        bound = conv_bound(xp, wt, st, p, dl)
    oh, ow = ref.shape[-2:]
    res = rnd(n, cout, oh, ow, seed=4)
    ncs = rnd(n, cout, seed=5, lo=0.5, hi=1.5)
    for variant in range(3):
        # 0: bias + lrelu ; 1: nc_scale + residual-before + sigmoid ; 2: residual-after + tanh + wide out slice
        y = NHWC.empty(n, oh, ow, cout + 5, DEV).slice(3, cout)
        kwargs = dict(force_tile=tile, force_splits=splits)
        exp = ref.clone()
        if variant == 0:
            kwargs.update(act=ops.ACT_LRELU, alpha=0.2)
            exp = F.leaky_relu(exp, 0.2)
        elif variant == 1:
            rv = nhwc(res.float())
            kwargs.update(act=ops.ACT_SIGMOID, res=rv, nc_scale=ncs.float().to(DEV))
            exp = torch.sigmoid((exp - bias[None, :, None, None]) * ncs[:, :, None, None] + bias[None, :, None, None]
                                + res)
        else:
            rv = nhwc(res.float())
            kwargs.update(act=ops.ACT_TANH, res=rv, res_after=True)
            exp = torch.tanh(exp) + res
        ops.conv2d(ctx, nhwc(x.float()), cw, y, **kwargs)
        got = to_nchw(y)
        err = (got - exp).abs()
        lim = REL[prec] * (bound + 1) + 1e-6
        if variant == 1:
            lim = lim * 1.5
        assert (err <= lim).all(), f"variant {variant}: max err {err.max():.3e}, rel {(err / lim).max():.2f}"


@pytest.mark.parametrize("cfg", [
    dict(n=2, cin=64, h=7, w=9, cout=96, k=3, pad=0, op=0),      # GPEN upsampling modconv (:262-276)
    dict(n=2, cin=32, h=6, w=6, cout=64, k=3, pad=1, op=1),      # DNet ADAINDecoderBlock (base_blocks.py:240-250)
    dict(n=1, cin=64, h=5, w=8, cout=40, k=4, pad=1, op=0),
    dict(n=2, cin=36, h=4, w=5, cout=33, k=3, pad=2, op=1),      # generic gather + negative class offsets
])
def test_conv_transpose_polyphase(ctx, prec, cfg):
    """Polyphase stride-2 ConvTranspose2d (one stride-1 conv per output parity class, strided
    output) against F.conv_transpose2d, with the prologue / epilogue pieces the engines use."""
    n, cin, h, w, cout, k, pad, op = (cfg[key] for key in ("n", "cin", "h", "w", "cout", "k", "pad", "op"))
    wt = rnd(cin, cout, k, k, seed=11) / math.sqrt(cin * k * k)
    bias = rnd(cout, seed=12)
    x = rnd(n, cin, h, w, seed=13)
    s = rnd(n, cin, seed=14, lo=0.5, hi=1.5)
    d = rnd(n, cout, seed=15, lo=0.5, hi=1.5)
    ref = F.conv_transpose2d(x * s[:, :, None, None], wt, None, 2, pad, output_padding=op)
    bound = conv_bound(x * s[:, :, None, None], wt, 2, pad, 1, True, op)
    cw = ConvW(wt.float(), bias.float(), DEV, transposed=True, stride=2, padding=pad, output_padding=op)
    cw.make_polyphase(DEV)
    oh, ow = ref.shape[-2:]
    assert cw.out_hw(h, w) == (oh, ow)
    exp = F.leaky_relu(ref * d[:, :, None, None] + bias[None, :, None, None], 0.2)
    y = NHWC.empty(n, oh, ow, cout + 4, DEV).slice(4, cout)
    ops.conv2d(ctx, nhwc(x.float()), cw, y, in_scale=s.float().to(DEV), nc_scale=d.float().to(DEV),
               act=ops.ACT_LRELU, alpha=0.2)
    err = (to_nchw(y) - exp).abs()
    lim = 2 * REL[prec] * (bound * 1.5 + 1) + 1e-6
    assert (err <= lim).all(), f"max err {err.max():.3e}"
    # in-place residual (DNet x_s + dx): y += conv_transpose(x)
    base = to_nchw(y)
    cw2 = ConvW(wt.float(), None, DEV, transposed=True, stride=2, padding=pad, output_padding=op).make_polyphase(DEV)
    ops.conv2d(ctx, nhwc(x.float()), cw2, y, res=y)
    ref2 = F.conv_transpose2d(x, wt, None, 2, pad, output_padding=op)
    err = (to_nchw(y) - (base + ref2)).abs()
    assert (err <= lim + 2 * REL[prec] * base.abs()).all(), f"residual max err {err.max():.3e}"


@pytest.mark.parametrize("n,h,w,c", [(2, 12, 12, 384), (3, 24, 24, 96), (2, 48, 48, 48), (1, 6, 10, 8)])
def test_rfft2_irfft2_match_torch_fft(ctx, n, h, w, c):
    """Separable LDS transforms (s2v_rfft2 / s2v_irfft2) against torch.fft.rfftn / irfftn ortho
    (ffc.py:99, :121), input a channel slice of a wider NHWC tensor, inverse with the residual."""
    x = rnd(n, h, w, c + 4, seed=21)
    wf = w // 2 + 1
    tables = ops.fft_tables(h, w, DEV)
    xin = NHWC(x.float().to(DEV)).slice(4, c)
    spec = torch.empty((n, h * wf, 2 * c), device=DEV)
    ops.rfft2(ctx, xin, tables, spec)
    ref = torch.fft.rfftn(x[..., 4:], dim=(1, 2), norm="ortho")              # [n, h, wf, c]
    got = spec.double().cpu().reshape(n, h, wf, 2, c)
    assert (got[..., 0, :] - ref.real).abs().max() < 2e-5 and (got[..., 1, :] - ref.imag).abs().max() < 2e-5
    sp = rnd(n, h * wf, 2 * c, seed=22)
    res = rnd(n, h, w, c, seed=23)
    y = NHWC.empty(n, h, w, c, DEV)
    ops.irfft2(ctx, sp.float().to(DEV), tables, y, res=NHWC(res.float().to(DEV)))
    z = sp.reshape(n, h, wf, 2, c)
    ref = torch.fft.irfftn(torch.complex(z[..., 0, :], z[..., 1, :]), s=(h, w), dim=(1, 2), norm="ortho") + res
    assert (y.t.double().cpu() - ref).abs().max() < 2e-5


@pytest.mark.parametrize("n,cin,h,w,cout,k,mode", [(3, 64, 10, 12, 96, 3, "direct"), (2, 4, 9, 9, 64, 3, "direct"),
                                                   (2, 32, 6, 6, 48, 3, "up2"), (2, 128, 7, 7, 3, 1, "direct")])
def test_modulated_conv_per_sample_weights(ctx, prec, n, cin, h, w, cout, k, mode):
    """s2v_modulate_weights + batched conv == the shared-weight form conv(x * s, W) * d (and the
    grouped per-sample conv of the reference, base_blocks.py:487-508)."""
    wt = rnd(cout, cin, k, k, seed=31) / math.sqrt(cin * k * k)
    bias = rnd(cout, seed=32)
    x = rnd(n, cin, h, w, seed=33)
    s = rnd(n, cin, seed=34, lo=0.5, hi=1.5)
    d = rnd(n, cout, seed=35, lo=0.5, hi=1.5)
    noise = rnd(n, 2 * h if mode == "up2" else h, 2 * w if mode == "up2" else w, seed=36)
    cw = ConvW(wt.float(), bias.float(), DEV, padding=k // 2,
               in_mode=ops.IN_NEAREST_UP2 if mode == "up2" else ops.IN_DIRECT)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if mode == "up2" else x
    wb = wt[None] * s[:, None, :, None, None] * d[:, :, None, None, None]
    ref = torch.stack([F.conv2d(xin[i:i + 1], wb[i], None, 1, k // 2)[0] for i in range(n)])
    ref = F.leaky_relu(ref + 0.3 * noise[:, None] + bias[None, :, None, None], 0.2)
    bound = conv_bound(xin * s[:, :, None, None], wt, 1, k // 2, 1) * 1.5 + 1
    oh, ow = ref.shape[-2:]
    y = NHWC.empty(n, oh, ow, cout + 4, DEV).slice(2, cout)
    ops.modulated_conv2d(ctx, nhwc(x.float()), cw, y, s.float().to(DEV), d.float().to(DEV), act=ops.ACT_LRELU,
                         alpha=0.2, pix_add=noise.float().to(DEV).contiguous(), pix_w=0.3)
    err = (to_nchw(y) - ref).abs()
    assert (err <= 2 * REL[prec] * bound + 1e-6).all(), f"max err {err.max():.3e}"
    # the modulation run ahead (ops.modulate_weights, engine/enet.py PREMOD) and read by the conv: bit-identical,
    # with and without the demodulation; a pre-modulated layout the conv does not read is refused.  (Cout <= 4
    # layers run the fp32 direct kernels, whose layout modulate_weights writes in f32 mode only.)
    for dd in ((d, None) if cout > 4 and cin > 4 else ()):     # (4-channel layers: exact fp32, conv_k4.hip)
        dv = None if dd is None else dd.float().to(DEV)
        kw = dict(act=ops.ACT_LRELU, alpha=0.2, pix_add=noise.float().to(DEV).contiguous(), pix_w=0.3)
        y1 = NHWC.empty(n, oh, ow, cout, DEV)
        ops.modulated_conv2d(ctx, nhwc(x.float()), cw, y1, s.float().to(DEV), dv, **kw)
        pm = ops.modulate_weights(ctx, cw, s.float().to(DEV), dv, n)
        y2 = NHWC.empty(n, oh, ow, cout, DEV)
        ops.modulated_conv2d(ctx, nhwc(x.float()), cw, y2, s.float().to(DEV), dv, premod=pm, **kw)
        torch.cuda.synchronize()
        assert torch.equal(y1.t, y2.t)
        with pytest.raises(Exception, match="pre-modulated"):
            ops.modulated_conv2d(ctx, nhwc(x.float()), cw, y2, s.float().to(DEV), dv, premod=(pm[0], -pm[1]), **kw)


@pytest.mark.parametrize("tile", [0, 4, 5, 6, 8, 9, 10, 11, 12])
@pytest.mark.parametrize("nhw", [(3, 10, 10), (2, 32, 32)])
def test_conv2d_prologue(ctx, prec, tile, nhw):
    """Input scale s[n, c] + pre-activation prologue on every tile family: the small tiles load s with
    the A operand (issue), the 256-row tiles one s pair per channel slice when the tile lies in one
    image, the wide ones in the store phase; 3 images of 10x10 (one tile spans several images: per-row
    image index) and 2 of 32x32 (every 256-row tile inside one image)."""
    if prec == "f32" and tile > 6:
        pytest.skip("the f32 table has 6 tiles")
    n, h, w = nhw
    cin, cout = 64, 64
    wt = rnd(cout, cin, 3, 3, seed=7) / math.sqrt(cin * 9)
    x = rnd(n, cin, h, w, seed=8)
    s = rnd(n, cin, seed=9, lo=0.5, hi=2.0)
    cw = ConvW(wt.float(), None, DEV, padding=1)
    y = NHWC.empty(n, h, w, cout, DEV)
    ops.conv2d(ctx, nhwc(x.float()), cw, y, in_scale=s.float().to(DEV), pre_act=ops.ACT_LRELU, pre_alpha=0.1,
               force_tile=tile)
    ref = F.conv2d(F.leaky_relu(x * s[:, :, None, None], 0.1), wt, padding=1)
    bound = conv_bound(F.leaky_relu(x * s[:, :, None, None], 0.1), wt, 1, 1, 1)
    assert ((to_nchw(y) - ref).abs() <= 2 * REL[prec] * (bound + 1) + 1e-6).all()


def test_gemm_kn_batched(ctx, prec):
    b, M, K, N = 3, 70, 144, 44
    a = rnd(M, K, seed=10).float()
    bm = rnd(b, K, N, seed=11).float()
    res = rnd(b, M, N, seed=12).float()
    out = torch.empty(b, M, N, device=DEV)
    ops.gemm_kn(ctx, a.to(DEV), bm.to(DEV), out, batch=b, a_bs=0, b_bs=K * N, out_bs=M * N, res=res.to(DEV),
                res_bs=M * N)
    ref = torch.einsum("mk,bkn->bmn", a.double(), bm.double()) + res.double()
    bound = torch.einsum("mk,bkn->bmn", a.double().abs(), bm.double().abs())
    assert ((out.double().cpu() - ref).abs() <= REL[prec] * (bound + 1) + 1e-6).all()


@pytest.mark.parametrize("c", [40, 42])                # float4 apply (pooled and not), scalar apply
@pytest.mark.parametrize("hw", [(12, 10), (18, 14)])
def test_layernorm2d(ctx, c, hw):
    h, w = hw
    x = rnd(2, c, h, w, seed=13) * 3 + 1
    wgt, b = rnd(c, seed=14), rnd(c, seed=15)
    xv = nhwc(x.float())
    for pool in (False, True):
        oh, ow = (h // 2, w // 2) if pool else (h, w)
        res = rnd(2, c, oh, ow, seed=16 + pool)
        y = NHWC.empty(2, oh, ow, c, DEV)
        ops.layernorm2d(ctx, xv, wgt.float().to(DEV), b.float().to(DEV), y, act=ops.ACT_LRELU, alpha=0.1, pool=pool,
                        res=nhwc(res.float()))
        ref = F.leaky_relu(F.layer_norm(x, x.shape[1:], wgt[:, None, None].expand(x.shape[1:]),
                                        b[:, None, None].expand(x.shape[1:]), 1e-5), 0.1)
        if pool:
            ref = F.avg_pool2d(ref, 2)
        assert (to_nchw(y) - (ref + res)).abs().max() < 2e-5


@pytest.mark.parametrize("strided", [False, True])
def test_layernorm2d_multiblock(ctx, strided):
    """Several statistics blocks per image (dense rows: the contiguous four-loads-in-flight reduction;
    a channel slice of a wider tensor: the strided one) and LN_EPT-step applies with ragged tails."""
    n, c, h, w = 2, 64, 66, 50
    x = rnd(n, c, h, w, seed=23) * 2 + 0.5
    wgt, b = rnd(c, seed=24), rnd(c, seed=25)
    if strided:
        wide = NHWC(torch.zeros(n, h, w, c + 8, device=DEV))
        wide.t[..., 4: 4 + c] = x.float().permute(0, 2, 3, 1).to(DEV)
        xv = wide.slice(4, c)
    else:
        xv = nhwc(x.float())
    for pool in (False, True):
        oh, ow = (h // 2, w // 2) if pool else (h, w)
        y = NHWC.empty(n, oh, ow, c, DEV)
        ops.layernorm2d(ctx, xv, wgt.float().to(DEV), b.float().to(DEV), y, act=ops.ACT_LRELU, alpha=0.2, pool=pool)
        ref = F.leaky_relu(F.layer_norm(x, x.shape[1:], wgt[:, None, None].expand(x.shape[1:]),
                                        b[:, None, None].expand(x.shape[1:]), 1e-5), 0.2)
        if pool:
            ref = F.avg_pool2d(ref, 2)
        assert (to_nchw(y) - ref).abs().max() < 2e-5


@pytest.mark.parametrize("c", [70, 72, 300])          # scalar path, float4 path, two 256-channel blocks
def test_instnorm_adain(ctx, c):
    for (h, w) in ((12, 12), (70, 40)):
        x = rnd(2, c, h, w, seed=17) * 2 - 0.5
        g, bt = rnd(2, c, seed=18), rnd(2, c, seed=19)
        gb = torch.cat([g, bt], 1).float().to(DEV)
        res = rnd(2, c, h, w, seed=20)
        y = NHWC.empty(2, h, w, c, DEV)
        ops.instnorm(ctx, nhwc(x.float()), y, gb[:, :c], gb[:, c:], act=ops.ACT_LRELU,
                     alpha=0.01, res=nhwc(res.float()))
        ref = F.leaky_relu(F.instance_norm(x, eps=1e-5) * (1 + g[:, :, None, None]) + bt[:, :, None, None], 0.01) + res
        assert (to_nchw(y) - ref).abs().max() < 2e-5
        if c % 4 == 0:
            # the padded second output (LNet FFC: the next block's reflect-padded 3x3 input): the same
            # values as y, laid out as F.pad(y, (1, 1, 1, 1), 'reflect'); y itself unchanged
            y2 = NHWC.empty(2, h, w, c, DEV)
            yp = NHWC(torch.full((2, h + 2, w + 2, c), float("nan"), device=DEV))
            ops.instnorm(ctx, nhwc(x.float()), y2, gb[:, :c], gb[:, c:], act=ops.ACT_LRELU,
                         alpha=0.01, res=nhwc(res.float()), pad_out=yp)
            assert torch.equal(y2.t, y.t)
            exp = F.pad(y.t.permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect").permute(0, 2, 3, 1)
            assert torch.equal(yp.t, exp)


def test_row_layernorm_attention(ctx):
    b, T, heads = 2, 144, 4
    x = rnd(b * T, 512, seed=21).float().to(DEV)
    wgt, bias = rnd(512, seed=22).float().to(DEV), rnd(512, seed=23).float().to(DEV)
    y = torch.empty_like(x)
    ops.row_layernorm(ctx, x, wgt, bias, y)
    ref = F.layer_norm(x.double().cpu(), (512,), wgt.double().cpu(), bias.double().cpu())
    assert (y.double().cpu() - ref).abs().max() < 2e-5
    qk = rnd(b * T, 512, seed=24).float().to(DEV)
    v = rnd(b * T, 256, seed=25).float().to(DEV)
    o = torch.empty(b * T, 256, device=DEV)
    ops.attention(ctx, qk[:, :256], qk[:, 256:], v, o, batch=b, heads=heads, tokens=T)
    q = qk[:, :256].double().cpu().reshape(b, T, heads, 64).transpose(1, 2)
    k = qk[:, 256:].double().cpu().reshape(b, T, heads, 64).transpose(1, 2)
    vv = v.double().cpu().reshape(b, T, heads, 64).transpose(1, 2)
    ref = (torch.softmax(q @ k.transpose(-1, -2) * 0.125, -1) @ vv).transpose(1, 2).reshape(b * T, 256)
    assert (o.double().cpu() - ref).abs().max() < 1e-5


@pytest.mark.parametrize("b,nh,L,total,contig", [(3, 128, 5, 300, False), (20, 100, 9, 1000, True),
                                                  (16, 128, 12, 4000, True), (2, 160, 3, 130, False),
                                                  (4, 512, 23, 1700, True), (3, 600, 2, 100, False)])
def test_adain_params_and_demod(ctx, b, nh, L, total, contig):
    """adain_heads2 (nh <= 128: 64-output blocks, 16-sample chunks, segment windows of 4; nh <= 512:
    one-segment windows — GFPGAN's per-layer style bank) and the v1 kernel (nh > 512); segments random
    per output or in contiguous runs as AdainBank / the GFPGAN bank lay them out."""
    hid = rnd(b, L * nh, seed=26).float().to(DEV)
    if contig:
        seg = (torch.arange(total) * L // total).int()
    else:
        seg = torch.randint(0, L, (total,), generator=torch.Generator().manual_seed(0)).int()
    w2 = rnd(total, nh, seed=27).float()
    bias = rnd(total, seed=28).float()
    out = torch.empty(b, total, device=DEV)
    ops.adain_params(ctx, hid, nh, w2.t().contiguous().to(DEV), bias.to(DEV), seg.to(DEV), out)
    h = hid.double().cpu().reshape(b, L, nh)
    ref = torch.stack([h[:, int(seg[o])] @ w2[o].double() for o in range(total)], 1) + bias.double()
    assert (out.double().cpu() - ref).abs().max() < 1e-4
    s = rnd(b, 40, seed=29).float().to(DEV)
    wsq = rnd(24, 40, seed=30, lo=0, hi=1).float().to(DEV)
    d = torch.empty(b, 24, device=DEV)
    ops.modconv_demod(ctx, s, wsq, d, eps=1e-8, post=math.sqrt(2))
    ref = torch.rsqrt((s.double().cpu() ** 2) @ wsq.double().cpu().t() + 1e-8) * math.sqrt(2)
    assert ((d.double().cpu() - ref).abs() / ref).max() < 1e-5


@pytest.mark.parametrize("b", [1, 4, 19])
def test_demod_rows_segmented(ctx, b):
    """ops.DemodRows: several layers' demodulations in one launch (ragged cin: one partial 64-lane
    chunk, a 256-wide chunk plus a tail, 1024; batch past the 16-sample chunk) against per-layer fp64."""
    shapes = [(24, 40), (33, 300), (16, 1024), (8, 512), (5, 7)]
    offs, o = [], 0
    for _, cin in shapes:
        offs.append(o)
        o += cin + 3
    s = rnd(b, o + 5, seed=31).float().to(DEV)
    ws = [rnd(co, ci, seed=32 + i, lo=0, hi=1).float() for i, (co, ci) in enumerate(shapes)]
    t = ops.DemodRows(list(zip(offs, ws)), DEV)
    d = torch.full((b, t.nrows + 6), -1.0, device=DEV)
    ops.modconv_demod_rows(ctx, s, t, d, eps=1e-8, post=math.sqrt(2))
    sd = s.double().cpu()
    for r0, off, w in zip(t.r0, offs, ws):
        ci = w.shape[1]
        ref = torch.rsqrt((sd[:, off: off + ci] ** 2) @ w.double().t() + 1e-8) * math.sqrt(2)
        got = d[:, r0: r0 + w.shape[0]].double().cpu()
        assert ((got - ref).abs() / ref).max() < 1e-5
    assert (d[:, t.nrows:] == -1).all()


@pytest.mark.parametrize("shape", [((2, 3, 384, 384), (96, 96), None), ((2, 5, 64, 64), None, 0.5),
                                   ((1, 4, 50, 50), None, 2), ((1, 3, 256, 256), (256, 256), None),
                                   ((2, 6, 100, 90), (37, 53), None), ((2, 8, 40, 36), None, 0.5),
                                   ((1, 16, 20, 20), None, 2)])
def test_resize_bilinear(ctx, shape):
    ishape, size, sf = shape
    x = rnd(*ishape, seed=31).float()
    ref = F.interpolate(x, size=size, scale_factor=sf, mode="bilinear", align_corners=False)
    y = NHWC.empty(ishape[0], ref.shape[2], ref.shape[3], ishape[1], DEV)
    ops.resize_nhwc(ctx, nhwc(x), y, scale_factor=sf)
    assert (to_nchw(y) - ref.double()).abs().max() < 2e-6
    y2 = NHWC.empty(ishape[0], ref.shape[2], ref.shape[3], ishape[1], DEV)
    ops.nchw_to_nhwc(ctx, x.to(DEV), y2) if sf is None else ops.resize_nhwc(ctx, nhwc(x), y2, scale_factor=sf)
    assert (to_nchw(y2) - ref.double()).abs().max() < 2e-6


@pytest.mark.parametrize("n,c,h,w,extra", [(2, 64, 7, 9, 0), (3, 4, 100, 100, 0), (1, 32, 13, 5, 8)])
def test_resize_up2_quads(ctx, n, c, h, w, extra):
    """Exact x2 upsample (2x2 output quads per thread: the StyleConv / ToRGB upsamples) against
    F.interpolate, into a channel slice of a wider output (edges clamp on every side)."""
    x = rnd(n, c, h, w, seed=33).float()
    ref = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    y = NHWC.empty(n, 2 * h, 2 * w, c + extra, DEV).slice(extra, c)
    ops.resize_nhwc(ctx, nhwc(x), y, scale_factor=2)
    assert (to_nchw(y) - ref.double()).abs().max() < 2e-6


def test_pad_reflect_and_crop(ctx):
    x = rnd(2, 3, 96, 96, seed=32).float()
    y = NHWC.empty(2, 100, 100, 3, DEV)
    ops.pad_reflect(ctx, nhwc(x), y, (2, 2, 2, 2))
    ref = F.pad(x, (2, 2, 2, 2), mode="reflect")
    assert torch.equal(to_nchw(y).float(), ref)
    out = torch.empty(2, 3, 84, 84, device=DEV)
    ops.nhwc_to_nchw(ctx, y, out, crop=(8, 8))
    assert torch.equal(out.cpu(), ref[:, :, 8:-8, 8:-8])


def test_flow_warp_matches_golden(ctx, golden):
    from s2v_amd import synth
    g = golden("ops")
    for key, fshape, sshape, name in (("golden.flow", (2, 2, 16, 16), (2, 3, 64, 64), "warp"),
                                      ("golden.flow2", (1, 2, 32, 32), (1, 3, 32, 32), "warp_same")):
        lo, hi = (-3.0, 3.0) if name == "warp" else (-2.0, 2.0)
        flow = torch.from_numpy(synth.hash_array(key, fshape, lo, hi))
        src = torch.from_numpy(synth.hash_array(key + ".src", sshape)).to(DEV)
        y = NHWC.empty(sshape[0], sshape[2], sshape[3], 3, DEV)
        ops.flow_warp(ctx, nhwc(flow), src, y)
        assert np.abs(to_nchw(y).numpy() - g[name]).max() < 2e-5


def test_gpen_ops_match_golden(ctx, golden):
    from s2v_amd import synth
    g = golden("ops")
    x = torch.from_numpy(synth.hash_array("golden.fba.x", (2, 8, 5, 7))).to(DEV)
    b = torch.from_numpy(synth.hash_array("golden.fba.b", (8,))).to(DEV)
    y = torch.empty_like(x)
    ops.check(ctx.lib.s2v_fused_bias_act(x.data_ptr(), b.data_ptr(), None, y.data_ptr(), x.numel(), 8, 35, 3, 0, 0.2,
                                         2 ** 0.5, ctx.stream), "fba")
    assert np.abs(y.cpu().numpy() - g["fba_out"]).max() < 1e-6
    xi = torch.from_numpy(synth.hash_array("golden.ufd.x", (2, 3, 9, 11))).to(DEV)
    k = torch.tensor([1.0, 3.0, 3.0, 1.0])
    k = (k[None, :] * k[:, None]) / 64.0
    for name, (up, down, pad) in {"up2": (2, 1, (2, 1)), "blur22": (1, 1, (2, 2)), "blur11": (1, 1, (1, 1)),
                                  "down2": (1, 2, (1, 1))}.items():
        kk = (k * (4 if up == 2 else 1)).to(DEV)
        exp = g[f"ufd_{name}"]
        oh, ow = exp.shape[-2:]
        out = torch.empty(6, oh, ow, 1, device=DEV)
        ops.check(ctx.lib.s2v_upfirdn2d(xi.data_ptr(), 6, 9, 11, 1, kk.data_ptr(), 4, 4, up, up, down, down, pad[0],
                                        pad[1], pad[0], pad[1], out.data_ptr(), oh, ow, ctx.stream), "upfirdn2d")
        assert np.abs(out.cpu().numpy().reshape(exp.shape) - exp).max() < 1e-6, name


def test_gaussian_noise_stats(ctx):
    y = torch.empty(1 << 20, device=DEV)
    ops.gaussian_noise(ctx, y, 1234)
    m, s = y.mean().item(), y.std().item()
    assert abs(m) < 5e-3 and abs(s - 1) < 5e-3
    y2 = torch.empty(1 << 20, device=DEV)
    ops.gaussian_noise(ctx, y2, 1234)
    assert torch.equal(y, y2)


def test_fourier_matrices_match_torch_fft(ctx):
    for h, w in ((12, 12), (24, 24), (48, 48)):
        d2, iv = ops.fourier_matrices(h, w, DEV)
        x = rnd(3, h, w, seed=33)
        spec = torch.fft.rfftn(x, dim=(-2, -1), norm="ortho")
        st = torch.stack([spec.real, spec.imag], -1).reshape(3, -1)
        got = (d2.double().cpu() @ x.reshape(3, -1).t()).t()
        assert (got - st).abs().max() < 1e-5
        back = (iv.double().cpu() @ st.t()).t().reshape(3, h, w)
        assert (back - x).abs().max() < 1e-5


@pytest.mark.parametrize("pad_mode", ["constant", "reflect"])
def test_melspectrogram_matches_restatement(pad_mode):
    """Device mel vs the float64 NumPy restatement of futils/audio.py (librosa 0.9.2 semantics;
    parity unpinned at the librosa boundary, see oracle/audio.py).  Tolerance 1e-3 in normalised
    units (range +-4), SURVEY.md §8d."""
    from oracle import audio as ref
    from s2v_amd import audio
    t = np.arange(48000) / 16000.0
    rng = np.random.default_rng(1)
    wav = (0.1 * rng.standard_normal(t.size) + 0.2 * (np.sin(2 * np.pi * 220 * t) + np.sin(2 * np.pi * 440 * t)
                                                         + np.sin(2 * np.pi * 1000 * t))).astype(np.float32)
    wav[:2000] = 0.0                                   # exercise the -100 dB floor / clip
    got = audio.melspectrogram(torch.from_numpy(wav).to(DEV), pad_mode=pad_mode).cpu().numpy()
    exp = ref.melspectrogram(wav, pad_mode=pad_mode)
    assert got.shape == exp.shape == (80, 241)
    assert np.abs(got - exp).max() < 1e-3
    chunks = audio.mel_chunks(torch.from_numpy(exp.astype(np.float32)).to(DEV)).cpu().numpy()
    starts = ref.mel_chunk_starts(exp.shape[1])
    assert chunks.shape == (len(starts), 1, 80, 16)
    for i, s in enumerate(starts):
        assert np.array_equal(chunks[i, 0], exp[:, s: s + 16].astype(np.float32))


@pytest.mark.parametrize("cin,k,cout", [(64, 7, 3), (128, 1, 3), (256, 1, 3), (256, 7, 2), (12, 3, 1),
                                        (32, 1, 3), (36, 3, 3), (44, 1, 2), (96, 3, 3)])
def test_small_cout_conv(ctx, prec, cin, k, cout):
    """Cout <= 4 heads (LNet/DNet final 7x7, ToRGB 1x1 with modulation, flow head): channel-parallel
    kernel with in_scale prologue and in-place residual.  cin 32..63 runs 2 lanes per pixel, 64..127
    4 lanes (36 / 44 leave the lanes' channel loops uneven), >= 128 8 lanes."""
    n, h, w = 2, 13, 11
    wt = rnd(cout, cin, k, k, seed=40) / math.sqrt(cin * k * k)
    bias = rnd(cout, seed=41)
    x = rnd(n, cin, h, w, seed=42)
    s = rnd(n, cin, seed=43, lo=0.5, hi=1.5)
    res = rnd(n, cout, h, w, seed=44)
    cw = ConvW(wt.float(), bias.float(), DEV, padding=k // 2)
    y = nhwc(res.float())
    ops.conv2d(ctx, nhwc(x.float()), cw, y, in_scale=s.float().to(DEV), res=y)
    ref = F.conv2d(x * s[:, :, None, None], wt, bias, padding=k // 2) + res
    bound = conv_bound(x * s[:, :, None, None], wt, 1, k // 2, 1)
    assert ((to_nchw(y) - ref).abs() <= 2e-6 * (bound + 1) + 1e-6).all()


@pytest.mark.parametrize("n,cin,h,w,k,cout,pad_mode,act", [
    (2, 64, 13, 11, 7, 3, "zero", ops.ACT_NONE),           # one strip, one band, partial everything
    (2, 64, 37, 130, 7, 3, "reflect", ops.ACT_TANH),      # DNet head form: 3 strips (58 + 58 + 14), 3 bands
    (3, 64, 96, 96, 7, 4, "zero", ops.ACT_SIGMOID),       # LNet head form (Cout carried as 4)
    (1, 32, 20, 64, 5, 4, "zero", ops.ACT_NONE),          # 5x5 over one 32-channel slice
    (2, 32, 9, 61, 7, 1, "reflect", ops.ACT_NONE),
    (2, 256, 20, 64, 7, 2, "zero", ops.ACT_NONE),          # DNet flow head form: 4 channel groups, split-K fold
    (1, 128, 9, 70, 5, 3, "reflect", ops.ACT_TANH),
    (2, 64, 5, 40, 7, 3, "reflect", ops.ACT_NONE)])        # 5 rows (odd band): the 2-row loop's unread extra
def test_conv_head_x3(ctx, prec, n, cin, h, w, k, cout, pad_mode, act):
    """Cout <= 4 wide-filter heads (conv_head.hip: kx in N, ky in K, an LDS ring of split input rows)
    in the split precisions; exact fp32 VALU (conv_halo_small / conv_small_cpar) in f32.  Against the
    fp64 conv at the per-mode bound of the implicit-GEMM kernels (REL * sum|a*b|)."""
    wt = rnd(cout, cin, k, k, seed=60) / math.sqrt(cin * k * k)
    bias = rnd(cout, seed=61)
    x = rnd(n, cin, h, w, seed=62, lo=-2.0, hi=2.0)
    pm = ops.PAD_REFLECT if pad_mode == "reflect" else ops.PAD_ZERO
    cw = ConvW(wt.float(), bias.float(), DEV, padding=k // 2, pad_mode=pm)
    y = NHWC.empty(n, h, w, cout, DEV)
    xd = nhwc(x.float())
    syms = []

    def hook(c, p, flops, launch):
        syms.append(ops.plan_symbol(p.plan))
        launch()
    ops.CONV_HOOK = hook
    try:
        ops.conv2d(ctx, xd, cw, y, act=act, alpha=0.0)
    finally:
        ops.CONV_HOOK = None
    if prec != "f32":
        assert syms and syms[0].startswith("void s2v::conv_head_x3<"), syms
    xp = F.pad(x, (k // 2,) * 4, mode="reflect") if pad_mode == "reflect" else x
    ref = F.conv2d(xp, wt, bias, padding=0 if pad_mode == "reflect" else k // 2)
    bound = conv_bound(xp, wt, 1, 0 if pad_mode == "reflect" else k // 2, 1)
    tol = (2e-6 if prec == "f32" else REL[prec]) * (bound + 1) + 1e-6
    got = to_nchw(y)
    if act == ops.ACT_TANH:
        ref = torch.tanh(ref)                             # |tanh'| <= 1
    elif act == ops.ACT_SIGMOID:
        ref, tol = torch.sigmoid(ref), tol / 4            # |sigmoid'| <= 1/4
    assert ((got - ref).abs() <= tol).all(), (got - ref).abs().max()


@pytest.mark.parametrize("n,hw,cin", [(2, (16, 8), 32), (2, (13, 11), 32), (3, (8, 16), 64), (2, (9, 7), 96)])
def test_small_cout_per_sample_weights(ctx, n, hw, cin):
    """Per-sample (modulated) weights on the small-Cout kernel: LDS-staged weights need every block
    inside one batch entry (M % pixels-per-block == 0, 16x8 = 128 pixels); other M take the global
    weight path.  Both against the grouped per-sample conv of the reference (base_blocks.py:487-508)."""
    h, w = hw
    cout = 3
    wt = rnd(cout, cin, 1, 1, seed=45) / math.sqrt(cin)
    bias = rnd(cout, seed=46)
    x = rnd(n, cin, h, w, seed=47)
    s = rnd(n, cin, seed=48, lo=0.5, hi=1.5)
    res = rnd(n, cout, h, w, seed=49)
    cw = ConvW(wt.float(), bias.float(), DEV)
    y = nhwc(res.float())
    ops.modulated_conv2d(ctx, nhwc(x.float()), cw, y, s.float().to(DEV), res=y)
    wb = wt[None] * s[:, None, :, None, None]
    ref = torch.stack([F.conv2d(x[i:i + 1], wb[i], bias)[0] for i in range(n)]) + res
    bound = conv_bound(x * s[:, :, None, None], wt, 1, 0, 1)
    assert ((to_nchw(y) - ref).abs() <= 2e-6 * (bound + 1) + 1e-6).all()


@pytest.mark.parametrize("n,h,w,cin", [(2, 16, 16, 256), (3, 32, 16, 128), (2, 8, 12, 64), (1, 40, 40, 32)])
def test_torgb_up2_fused(ctx, n, h, w, cin):
    """ToRGB + skip upsample in one pass (ops.torgb_up2, base_blocks.py:536-554) against the reference
    composition: per-sample 1x1 conv of W * s (no demodulation) + bias + F.interpolate(skip, x2,
    bilinear); the 4th channel is the upsampled skip's 4th.  Pixel counts cover every PPT variant."""
    wt = rnd(3, cin, 1, 1, seed=61) / math.sqrt(cin)
    bias = rnd(3, seed=62)
    x = rnd(n, cin, h, w, seed=63)
    s = rnd(n, cin, seed=64, lo=0.5, hi=1.5)
    skip = rnd(n, 4, h // 2, w // 2, seed=65)
    cw = ConvW(wt.float(), bias.float(), DEV)
    y = NHWC.empty(n, h, w, 4, DEV)
    ops.torgb_up2(ctx, nhwc(x.float()), cw, s.float().to(DEV), nhwc(skip.float()), y)
    up = F.interpolate(skip, scale_factor=2, mode="bilinear", align_corners=False)
    wb = wt[None] * s[:, None, :, None, None]
    conv = torch.stack([F.conv2d(x[i:i + 1], wb[i], bias)[0] for i in range(n)])
    ref = torch.cat([conv + up[:, :3], up[:, 3:]], 1)
    bound = torch.cat([conv_bound(x * s[:, :, None, None], wt, 1, 0, 1), up[:, 3:].abs()], 1) + up.abs()
    assert ((to_nchw(y) - ref).abs() <= 2e-6 * (bound + 1) + 1e-6).all()


@pytest.mark.parametrize("n,cin,h,w,cout", [(2, 64, 9, 7, 32), (3, 32, 12, 16, 128), (2, 4, 10, 12, 64)])
def test_modulated_conv_d2s_polyphase(ctx, prec, n, cin, h, w, cout):
    """x2-bilinear-upsample + modulated 3x3 conv as one depth-to-space conv over the un-upsampled
    input with the four folded parity-class filters (engine.enet.fold_up2_conv3, s2v_conv_params
    .d2s_cout) against the reference order (F.interpolate, then the per-sample conv + noise + bias +
    LeakyReLU, base_blocks.py:500-533), away from the two outermost output lines of each side (the
    engine recomputes those directly; tests/test_models_gpu.py covers the composed frame)."""
    from s2v_amd.engine.enet import fold_up2_conv3
    wt = rnd(cout, cin, 3, 3, seed=71) / math.sqrt(cin * 9)
    bias = rnd(cout, seed=72)
    x = rnd(n, cin, h, w, seed=73)
    s = rnd(n, cin, seed=74, lo=0.5, hi=1.5)
    d = rnd(n, cout, seed=75, lo=0.5, hi=1.5)
    noise = rnd(n, 2 * h, 2 * w, seed=76)
    cw4 = ConvW(fold_up2_conv3(wt.float()), bias.float().repeat(4), DEV, padding=1)
    y = NHWC.empty(n, 2 * h, 2 * w, cout, DEV)
    ops.modulated_conv2d(ctx, nhwc(x.float()), cw4, y, s.float().to(DEV), d.float().repeat(1, 4).to(DEV),
                         act=ops.ACT_LRELU, alpha=0.2, pix_add=noise.float().to(DEV), pix_w=0.3, d2s=True)
    up = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    wb = wt[None] * s[:, None, :, None, None] * d[:, :, None, None, None]
    conv = torch.stack([F.conv2d(up[i:i + 1], wb[i], bias, padding=1)[0] for i in range(n)])
    ref = F.leaky_relu(conv + 0.3 * noise[:, None], 0.2)
    bound = torch.stack([F.conv2d(up[i:i + 1].abs(), wb[i].abs(), padding=1)[0] for i in range(n)]) + 1
    err = (to_nchw(y) - ref).abs()[:, :, 2:-2, 2:-2]
    assert (err <= 4 * REL[prec] * bound[:, :, 2:-2, 2:-2] + 1e-6).all(), f"max err {err.max():.3e}"


@pytest.mark.parametrize("mag", [1e-2, 30.0])
def test_f16x3_operand_range(ctx, mag):
    """f16x3 keeps its 3 * 2^-22 per-product bound away from unit scale: activations of magnitude
    1e-2 (their lo halves are f16 subnormals: a flushing MFMA would lose 2^-12 of each) and 30 (weights
    pre-scaled by a power of two, undone in the epilogue), weights scaled by 1 / mag."""
    prev = ops.set_precision("f16x3")
    try:
        n, cin, h, w, cout = 2, 64, 12, 12, 96
        wt = rnd(cout, cin, 3, 3, seed=51) / math.sqrt(cin * 9) / mag
        x = rnd(n, cin, h, w, seed=52) * mag
        cw = ConvW(wt.float(), None, DEV, padding=1)
        y = NHWC.empty(n, h, w, cout, DEV)
        ops.conv2d(ctx, nhwc(x.float()), cw, y)
        ref = F.conv2d(x.float().double(), wt.float().double(), padding=1)
        bound = conv_bound(x.float().double(), wt.float().double(), 1, 1, 1)
        err = (to_nchw(y) - ref).abs()
        assert (err <= REL["f16x3"] * bound + 1e-12).all(), f"max rel {(err / (bound + 1e-30)).max():.3e}"
    finally:
        ops.set_precision(prev)


@pytest.mark.parametrize("n,cin,h,w,cout,tile", [(2, 64, 12, 16, 96, 0), (2, 32, 8, 8, 64, 5), (1, 256, 16, 16, 256, 1),
                                                 (3, 4, 10, 6, 40, 0), (2, 64, 6, 10, 48, 8),
                                                 (2, 64, 12, 16, 96, 10), (1, 32, 10, 14, 32, 11)])
def test_conv2d_pooled_epilogue(ctx, prec, n, cin, h, w, cout, tile):
    """out_pool: the 2x2 mean of lrelu(conv + b) (ResBlock conv1 + bilinear x0.5, base_blocks.py:40-49)
    written at half size; M runs over 2x2 quads, so every tile holds whole quads."""
    if tile > 6 and prec == "f32":
        pytest.skip("tiles 7-12 exist in the split-precision table only")
    wt = rnd(cout, cin, 3, 3, seed=61) / math.sqrt(cin * 9)
    bias = rnd(cout, seed=62)
    x = rnd(n, cin, h, w, seed=63)
    cw = ConvW(wt.float(), bias.float(), DEV, padding=1)
    y = NHWC.empty(n, h // 2, w // 2, cout + 3, DEV).slice(1, cout)
    ops.conv2d(ctx, nhwc(x.float()), cw, y, act=ops.ACT_LRELU, alpha=0.2, pool=True, force_tile=tile)
    full = F.leaky_relu(F.conv2d(x, wt, bias, 1, 1), 0.2)
    ref = F.interpolate(full, scale_factor=0.5, mode="bilinear", align_corners=False)
    bound = F.avg_pool2d(conv_bound(x, wt, 1, 1, 1), 2)
    err = (to_nchw(y) - ref).abs()
    assert (err <= REL[prec] * (bound + 1) + 1e-6).all(), f"max err {err.max():.3e}"


def test_resblock_skip_as_strided_conv(ctx, prec):
    """skip(interpolate(x, 0.5)) of a 1x1 conv == a 2x2 stride-2 conv with W / 4 on each tap
    (engine/enet.py): against the reference order of operations."""
    n, cin, h, w, cout = 2, 64, 12, 10, 96
    wt = rnd(cout, cin, 1, 1, seed=64) / math.sqrt(cin)
    x = rnd(n, cin, h, w, seed=65)
    cw = ConvW((wt.float() / 4).expand(-1, -1, 2, 2).contiguous(), None, DEV, stride=2)
    y = NHWC.empty(n, h // 2, w // 2, cout, DEV)
    ops.conv2d(ctx, nhwc(x.float()), cw, y)
    ref = F.conv2d(F.interpolate(x, scale_factor=0.5, mode="bilinear", align_corners=False), wt)
    bound = F.conv2d(F.avg_pool2d(x.abs(), 2), wt.abs())
    assert ((to_nchw(y) - ref).abs() <= REL[prec] * (bound + 1) + 1e-6).all()


@pytest.mark.parametrize("n,c,h,w", [(16, 1024, 12, 12), (16, 256, 24, 24), (3, 40, 10, 9)])
def test_instnorm_fused_small_planes(ctx, n, c, h, w):
    """LNet's 12^2 / 24^2 planes (and a ragged one): one-launch InstanceNorm (S2V_TUNE_IN_FUSED = max
    plane pixels, narrow channel groups) against the two-pass form and torch, with the residual and
    the reflect-padded second output."""
    x = rnd(n, c, h, w, seed=31) * 2 - 0.5
    g, bt = rnd(n, c, seed=32), rnd(n, c, seed=33)
    gb = torch.cat([g, bt], 1).float().to(DEV)
    res = rnd(n, c, h, w, seed=34)
    outs = {}
    for fused in (1, 0):
        prev = ops.tune(ctx, ops.TUNE_IN_FUSED, h * w if fused else 0)
        try:
            y = NHWC.empty(n, h, w, c, DEV)
            yp = NHWC.empty(n, h + 2, w + 2, c, DEV)
            ops.instnorm(ctx, nhwc(x.float()), y, gb[:, :c], gb[:, c:], act=ops.ACT_LRELU,
                         alpha=0.01, res=nhwc(res.float()), pad_out=yp)
            outs[fused] = (y.t.clone(), yp.t.clone())
        finally:
            ops.tune(ctx, ops.TUNE_IN_FUSED, prev)
    ref = F.leaky_relu(F.instance_norm(x, eps=1e-5) * (1 + g[:, :, None, None]) + bt[:, :, None, None], 0.01) + res
    y1, p1 = outs[1]
    assert (y1.permute(0, 3, 1, 2).cpu() - ref).abs().max() < 2e-5
    assert (y1 - outs[0][0]).abs().max() < 1e-5
    assert torch.equal(p1, F.pad(y1.permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect").permute(0, 2, 3, 1))


@pytest.mark.parametrize("tile,splits,cap", [(1, 0, 8), (1, 0, 24), (1, 2, 16), (4, 3, 40)])
def test_conv_x3_grid_cap_bit_exact(ctx, tile, splits, cap):
    """s2v_conv_params.grid_cap (ops.x3_grid_cap, per context): ``cap`` persistent blocks looping over
    the tile grid (more tiles than blocks, a ragged last round) compute every tile exactly as the
    one-block-per-tile launch does — same K order, same epilogue — so the outputs are bit-identical (with
    and without split-K); both are checked against the fp64 reference at the f16x3 bound.  The persistent
    kernel exists for the 256x256 tile (force_tile 1) and the plan says it is taken; other tiles ignore
    the cap (force_tile 4)."""
    n, cin, h, w, cout = 2, 64, 64, 64, 160
    wt = rnd(cout, cin, 3, 3, seed=11) / math.sqrt(cin * 9)
    bias = rnd(cout, seed=12)
    cw = ConvW(wt.float(), bias.float(), DEV, padding=1)
    x = rnd(n, cin, h, w, seed=13)
    prev_p = ops.set_precision("f16x3")
    try:
        outs, syms = [], []
        for c in (0, cap):
            with ops.x3_grid_cap(ctx, c):
                y = NHWC.empty(n, h, w, cout, DEV)
                ops.conv2d(ctx, nhwc(x.float()), cw, y, act=ops.ACT_LRELU, alpha=0.2, force_tile=tile,
                           force_splits=splits)
                outs.append(y)
                seen = {}

                def hook(c_, p, flops, launch):
                    seen["plan"] = p.plan
                    launch()
                ops.CONV_HOOK = hook
                try:
                    ops.conv2d(ctx, nhwc(x.float()), cw, NHWC.empty(n, h, w, cout, DEV), force_tile=tile,
                               force_splits=splits)
                finally:
                    ops.CONV_HOOK = None
                syms.append((seen["plan"][10], ops.plan_symbol(seen["plan"])))
        assert ctx.grid_cap == 0
    finally:
        ops.set_precision(prev_p)
    assert syms[0][0] == 0 and "persist" not in syms[0][1]
    if tile == 1:
        assert syms[1][0] == cap and syms[1][1].startswith("void s2v::conv_igemm_x3_persist<256, 256,"), syms[1]
    else:
        assert syms[1][0] == 0 and "persist" not in syms[1][1]
    assert torch.equal(outs[0].t, outs[1].t)
    ref = F.leaky_relu(F.conv2d(x, wt, bias, padding=1), 0.2)
    lim = REL["f16x3"] * (conv_bound(x, wt, 1, 1, 1) + 1) + 1e-6
    assert ((to_nchw(outs[1]) - ref).abs() <= lim).all()


@pytest.mark.parametrize("sprec", ["f16x3", "bf16x3"])
def test_conv_group_matches_reference(ctx, sprec):
    """s2v_conv2d_group (ops.conv_group): LNet's FFC fork as one launch — a K-heavy 3x3 valid conv, a
    wide 3x3 on a channel slice and a 1x1 with a BN-style epilogue + ReLU on another slice of the same
    input, each with its own split-K factor — against fp64 references at the split-precision bound,
    and the grouped plan really forms one group."""
    n, h, w = 2, 12, 12
    cin, cl = 256, 64
    x = rnd(n, cin, h + 2, w + 2, seed=71)                 # pre-padded block input
    xin = rnd(n, cin, h, w, seed=72)
    w1 = rnd(64, cin, 3, 3, seed=73) / math.sqrt(cin * 9)
    w2 = rnd(192, cl, 3, 3, seed=74) / math.sqrt(cl * 9)
    w3 = rnd(96, cin - cl, 1, 1, seed=75) / math.sqrt(cin - cl)
    sc, sh = rnd(96, seed=76, lo=0.5, hi=1.5), rnd(96, seed=77)
    cw1 = ConvW(w1.float(), None, DEV)
    cw2 = ConvW(w2.float(), None, DEV)
    cw3 = ConvW(w3.float(), None, DEV, post_scale=sc.float())
    cw3.shift = (sh.float()).to(DEV)
    prev = ops.set_precision(sprec)
    try:
        xp, xi = nhwc(x.float()), nhwc(xin.float())
        y = NHWC.empty(n, h, w, 256, DEV)
        t = NHWC.empty(n, h, w, 96, DEV)
        with ops.conv_group(ctx):
            ops.conv2d(ctx, xp, cw1, y.slice(0, 64))
            ops.conv2d(ctx, xp.slice(0, cl), cw2, y.slice(64, 192))
            ops.conv2d(ctx, xi.slice(cl, cin - cl), cw3, t, act=ops.ACT_RELU)
        torch.cuda.synchronize()
        params = []
        for xv, cw, yv in ((xp, cw1, y.slice(0, 64)), (xp.slice(0, cl), cw2, y.slice(64, 192)),
                           (xi.slice(cl, cin - cl), cw3, t)):
            p = _params_of(ctx, xv, cw, yv)
            params.append(p)
        arr = (ops._lib.ConvParams * 3)(*params)
        out = (ctypes.c_int * 5)()
        assert ctx.lib.s2v_conv2d_group_plan(arr, 3, out) == 0, ctx.lib.s2v_last_error()
        assert ops.LAST_GROUP == 1                        # the launch above was one grouped kernel
    finally:
        ops.set_precision(prev)
    r1 = F.conv2d(x, w1)
    r2 = F.conv2d(x[:, :cl], w2)
    r3 = F.relu(F.conv2d(xin[:, cl:], w3) * sc[None, :, None, None] + sh[None, :, None, None])
    for got, ref, bound in ((to_nchw(y.slice(0, 64)), r1, conv_bound(x, w1, 1, 0, 1)),
                            (to_nchw(y.slice(64, 192)), r2, conv_bound(x[:, :cl], w2, 1, 0, 1)),
                            (to_nchw(t), r3, conv_bound(xin[:, cl:], w3, 1, 0, 1) * sc.abs()[None, :, None, None])):
        err = (got - ref).abs()
        assert (err <= REL[sprec] * (bound + 1) + 1e-6).all(), f"max err {err.max():.3e}"


def _params_of(ctx, x, cw, y):
    """s2v_conv_params of a plain conv2d launch (ctypes), for the C ABI plan calls."""
    p = ops._lib.ConvParams()
    p.x, p.n, p.h, p.w, p.cin, p.xcs = x.ptr, x.n, x.h, x.w, x.c, x.cs
    p.kh, p.kw, p.sh, p.sw, p.ph, p.pw, p.dh, p.dw = cw.kh, cw.kw, cw.sh, cw.sw, cw.ph, cw.pw, cw.dh, cw.dw
    p.wt, p.kpad, p.npad, p.cout = cw.wt.data_ptr(), cw.kpad, cw.npad, cw.cout
    p.y, p.oh, p.ow, p.ycs = y.ptr, y.h, y.w, y.cs
    p.prec = ops.prec_code()
    p.wt_x3 = cw.wt_x3(ctx, p.prec).data_ptr()
    p.batch = 1
    return p


@pytest.mark.parametrize("sprec", ["f16x3", "bf16x3", "f32"])
@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 12, 12, 256, 64), (1, 20, 17, 64, 96), (4, 48, 48, 64, 32)])
def test_conv_up2_polyphase_matches_reference(ctx, sprec, n, h, w, cin, cout):
    """ConvW.make_up2_polyphase (UpBlock2d: nearest x2 then 3x3 zero-padded conv) as four parity-class 2x2
    convs of the un-upsampled input, grouped into one launch for small inputs, against fp64
    F.interpolate(nearest) + F.conv2d with bias: the whole output including the zero-padded borders
    and odd / even image sizes."""
    x = rnd(n, cin, h, w, seed=81)
    wt = rnd(cout, cin, 3, 3, seed=82) / math.sqrt(cin * 9)
    b = rnd(cout, seed=83)
    cw = ConvW(wt.float(), b.float(), DEV, padding=1, in_mode=ops.IN_NEAREST_UP2).make_up2_polyphase(DEV)
    prev = ops.set_precision(sprec)
    try:
        y = NHWC.empty(n, 2 * h, 2 * w, cout, DEV)
        ops.conv2d(ctx, nhwc(x.float()), cw, y)
        torch.cuda.synchronize()
        grouped = ops.LAST_GROUP
    finally:
        ops.set_precision(prev)
    xu = F.interpolate(x, scale_factor=2, mode="nearest")
    ref = F.conv2d(xu, wt, b, padding=1)
    err = (to_nchw(y) - ref).abs()
    bound = conv_bound(xu, wt, 1, 1, 1)
    assert (err <= REL[sprec] * (bound + 1) + 1e-6).all(), f"max err {err.max():.3e}"
    if sprec != "f32" and n * h * w <= ops.UP2_GROUP_PIXELS:
        assert grouped == 1                                # the four classes went out as one grouped launch


@pytest.mark.parametrize("sprec", ["f16x3", "bf16x3", "f32"])
@pytest.mark.parametrize("n,h,w,cin,cout,k,sl", [(2, 20, 23, 3, 64, 7, True), (3, 17, 16, 6, 64, 7, False),
                                                 (1, 9, 9, 8, 32, 5, False)])
def test_conv_rowpack_matches_reference(ctx, sprec, n, h, w, cin, cout, k, sl):
    """ConvW.make_rowpack (7x7 / 5x5 over <= 8 channels as a kh x 1 conv over row-tap packed channels,
    ops.row_pack) with bias + LeakyReLU, on a channel slice of a wider tensor (LNet's face6[..., :3]) or a
    dense input, against fp64 F.conv2d; and row_pack's layout itself (zero past the row and past kw*c)."""
    xt = rnd(n, 2 * cin if sl else cin, h, w, seed=91)
    wt = rnd(cout, cin, k, k, seed=92) / math.sqrt(cin * k * k)
    b = rnd(cout, seed=93)
    cw = ConvW(wt.float(), b.float(), DEV, padding=k // 2).make_rowpack(DEV)
    xv = nhwc(xt.float())
    xin = xv.slice(cin, cin) if sl else xv
    xr = xt[:, cin:] if sl else xt
    prev = ops.set_precision(sprec)
    try:
        y = NHWC.empty(n, h, w, cout, DEV)
        ops.conv2d(ctx, xin, cw, y, act=ops.ACT_LRELU, alpha=0.1)
        packed = NHWC.empty(n, h, w, cw.rowpack.cin, DEV)
        ops.row_pack(ctx, xin, packed, k, k // 2)
        torch.cuda.synchronize()
    finally:
        ops.set_precision(prev)
    ref = F.leaky_relu(F.conv2d(xr, wt, b, padding=k // 2), 0.1)
    err = (to_nchw(y) - ref).abs()
    bound = conv_bound(xr, wt, 1, k // 2, 1)
    assert (err <= REL[sprec] * (bound + 1) + 1e-6).all(), f"max err {err.max():.3e}"
    xp = F.pad(xr, (k // 2, k // 2))                                    # [n, c, h, w + k - 1]
    want = torch.zeros(n, h, w, cw.rowpack.cin, dtype=torch.float64)
    for dx in range(k):
        want[..., dx * cin:(dx + 1) * cin] = xp[:, :, :, dx:dx + w].permute(0, 2, 3, 1)
    assert torch.equal(packed.t.double().cpu(), want.float().double())


@pytest.mark.parametrize("cin,cout,tile", [(48, 96, 0), (40, 64, 4), (24, 48, 5), (8, 32, 0), (48, 256, 1), (72, 128, 11)])
def test_conv1x1_partial_slice_buffer_path(ctx, prec, cin, cout, tile):
    """1x1 convs over cin % 8 == 0 but not % 32 channels (LNet's 48^2 st2: 48 channels) on the buffer-load
    x3 path with a partial last K-slice (lanes past cin load zeros), on a channel slice of a wider tensor,
    with residual + bias + act, split-K, against fp64 F.conv2d."""
    if prec == "f32" and tile > 6:
        pytest.skip("the f32 table has 6 tiles")
    n, h, w = 2, 19, 23
    x = rnd(n, cin + 8, h, w, seed=101)
    wt = rnd(cout, cin, 1, 1, seed=102) / math.sqrt(cin)
    b = rnd(cout, seed=103)
    r = rnd(n, cout, h, w, seed=104)
    cw = ConvW(wt.float(), b.float(), DEV)
    xv = nhwc(x.float()).slice(8, cin)
    y = NHWC.empty(n, h, w, cout, DEV)
    rv = nhwc(r.float())
    ops.conv2d(ctx, xv, cw, y, act=ops.ACT_LRELU, alpha=0.2, res=rv, force_tile=tile,
               force_splits=2 if cin > 32 else 0)
    xr = x[:, 8:]
    ref = F.leaky_relu(F.conv2d(xr, wt, b) + r, 0.2)
    err = (to_nchw(y) - ref).abs()
    bound = conv_bound(xr, wt, 1, 0, 1)
    assert (err <= REL[prec] * (bound + 1) + 1e-5).all(), f"max err {err.max():.3e}"


def test_f16_split_variants_bit_identical():
    """the widen-subtract-pack f16 split (X3_F16_MIX=0) and the v_fma_mix split the
    library uses (1) give bit-identical hi / lo halves (s2v_f16_split_check runs both on the same inputs):
    normals over 14 decades down into the f16-subnormal lo range, and random fp32 bit patterns inside the
    f16 range.  (The r04 failure of 0 was the compiler re-converting the inputs for the widening instead of
    widening the stored hi halves; conv_x3_impl.hpp X3_F16_MIX.)"""
    from s2v_amd import _lib
    lib = _lib.load()
    g = torch.Generator().manual_seed(3)
    parts = [torch.randn(1 << 18, generator=g) * 10.0 ** e for e in range(-9, 5)]
    bits = torch.randint(0, 2 ** 31 - 1, (1 << 20,), generator=g, dtype=torch.int64).to(torch.int32).view(torch.float32)
    bits = bits[torch.isfinite(bits) & (bits.abs() < 6.0e4)]
    x = torch.cat(parts + [bits, -bits])
    x = x[x.abs() < 6.0e4]
    x = x[: x.numel() // 4 * 4].contiguous().to(DEV)
    m = torch.zeros(1, dtype=torch.int32, device=DEV)
    rc = lib.s2v_f16_split_check(x.data_ptr(), x.numel(), m.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, lib.s2v_last_error()
    torch.cuda.synchronize()
    assert int(m.item()) == 0, f"{int(m.item())} of {x.numel() // 4} float4s differ"


@pytest.mark.parametrize("tile,splits", [(0, 0), (1, 0), (4, 0), (4, 3), (8, 0), (11, 0), (18, 0), (18, 2), (20, 0)])
@pytest.mark.parametrize("nc", [False, True])
def test_conv2d_post_and_dup_epilogue(ctx, prec, tile, splits, nc):
    """The epilogue extras of the enhancers' StyleConvs, against fp64: ``post`` (GFPGAN's SFT on the
    upper half of the channels after the activation, gfpganv1_clean_arch.py:98-106) and ``dup`` (GPEN's
    noise-injection concat half as a second output beside the conv's, gpen_model.py:292-302), with and
    without the per-(image, channel) demodulation scale, through the LDS tiles, split-K (the split-K fold's
    epilogue) and the halo tile."""
    if tile > 6 and prec == "f32":
        pytest.skip("tiles 7-20 exist in the split-precision table only")
    n, cin, h, w, cout = 2, 64, 8, 64, 256 if tile == 1 else 64       # (the 256x256 tile needs 256 channels)
    c0 = cout // 2
    wt = rnd(cout, cin, 3, 3, seed=71) / math.sqrt(cin * 9)
    bias = rnd(cout, seed=72)
    x = rnd(n, cin, h, w, seed=73)
    d = rnd(n, cout, seed=74, lo=0.5, hi=1.5)
    pm, pa = rnd(n, cout - c0, h, w, seed=75), rnd(n, cout - c0, h, w, seed=76)
    ds, db = rnd(n, cout, h, w, seed=77), rnd(cout, seed=78)
    cw = ConvW(wt.float(), bias.float(), DEV, padding=1)
    full = NHWC.empty(n, h, w, 2 * cout, DEV)
    y = full.slice(0, cout)
    ops.conv2d(ctx, nhwc(x.float()), cw, y, act=ops.ACT_LRELU, alpha=0.2,
               nc_scale=d.float().to(DEV) if nc else None, force_tile=tile, force_splits=splits,
               post=(nhwc(pm.float()), nhwc(pa.float()), c0),
               dup=(nhwc(ds.float()), db.float().to(DEV), 0.7, cout))
    scale = d[:, :, None, None] if nc else torch.ones(1, cout, 1, 1, dtype=torch.float64)
    v = F.leaky_relu(F.conv2d(x, wt, padding=1) * scale + bias[None, :, None, None], 0.2)
    bound = conv_bound(x, wt, 1, 1, 1) * scale.abs()
    v[:, c0:] = v[:, c0:] * pm + pa
    bound[:, c0:] = bound[:, c0:] * pm.abs()
    got = to_nchw(full)
    err = (got[:, :cout] - v).abs()
    assert (err <= REL[prec] * (bound + 1) + 1e-6).all(), f"main: max err {err.max():.3e}"
    dref = F.leaky_relu(0.7 * ds + db[None, :, None, None], 0.2)
    assert (got[:, cout:] - dref).abs().max() < 1e-6


@pytest.mark.parametrize("n,h,w,cout,k,noise", [(3, 7, 9, 32, 3, False), (2, 16, 16, 96, 3, True),
                                                 (2, 20, 24, 256, 3, True), (3, 11, 13, 64, 1, False),
                                                 (1, 33, 40, 256, 1, True)])
def test_conv_k4_exact_fp32(ctx, prec, n, h, w, cout, k, noise):
    """4-channel "same" convs run on conv_k4_mfma (csrc/conv_k4.hip) in every precision mode, in exact fp32 (MFMA
    v_mfma_f32_32x32x2f32): against fp64 at the fp32 bound, including partial last tiles (h*w not a multiple of 32),
    Cout of one / three / eight 32-channel blocks, bias + noise + LeakyReLU in the epilogue, and the plan names the
    kernel."""
    wt = rnd(cout, 4, k, k, seed=81) / math.sqrt(4 * k * k)
    bias = rnd(cout, seed=82)
    x = rnd(n, 4, h, w, seed=83)
    nz = rnd(n, h, w, seed=84)
    cw = ConvW(wt.float(), bias.float(), DEV, padding=k // 2)
    seen = {}

    def hook(c_, p, flops, launch):
        seen["plan"] = p.plan
        launch()
    ops.CONV_HOOK = hook
    try:
        y = NHWC.empty(n, h, w, cout + 8, DEV).slice(4, cout)
        kw = dict(pix_add=nz.float().to(DEV).contiguous(), pix_w=0.3) if noise else {}
        ops.conv2d(ctx, nhwc(x.float()), cw, y, act=ops.ACT_LRELU, alpha=0.2, **kw)
    finally:
        ops.CONV_HOOK = None
    assert ops.plan_symbol(seen["plan"]).startswith("void s2v::conv_k4_mfma<"), ops.plan_symbol(seen["plan"])
    ref = F.conv2d(x, wt, bias, padding=k // 2) + (0.3 * nz[:, None] if noise else 0)
    ref = F.leaky_relu(ref, 0.2)
    err = (to_nchw(y) - ref).abs()
    assert (err <= REL["f32"] * (conv_bound(x, wt, 1, k // 2, 1) + 1) + 1e-6).all(), f"max err {err.max():.3e}"
