"""PyTorch custom ops (TORCH_LIBRARY(s2v), csrc/torch_ops.cpp) on the device.

* The GPEN native-op drop-ins with the exact call forms of the reference (gpen_model.py:54 Upsample,
  :76 Downsample, :96 Blur, :162 EqualLinear + fused_leaky_relu; op/fused_act.py:60-66,
  op/upfirdn2d.py:114-124) against tests/golden/ops.npz — outputs of the reference's own CPU
  fallbacks (fused_leaky_relu / upfirdn2d_native).
* The model-path ops against fp64 / torch references and against the ctypes engine path (same
  kernels, so bit-identical where the launch is identical).
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import s2v_import  # noqa: F401
from s2v_amd import ops, synth, torch_ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _blur_kernel(up):
    k = torch.tensor([1.0, 3.0, 3.0, 1.0])
    k = (k[None, :] * k[:, None]) / 64.0
    return (k * (4 if up == 2 else 1)).to(DEV)      # make_kernel, Upsample's factor**2 (gpen_model.py:37-44)


def test_gpen_call_forms_match_reference_goldens(golden):
    g = golden("ops")
    x = torch.from_numpy(synth.hash_array("golden.fba.x", (2, 8, 5, 7))).to(DEV)
    b = torch.from_numpy(synth.hash_array("golden.fba.b", (8,))).to(DEV)
    # FusedLeakyReLU.forward -> fused_leaky_relu (fused_act.py:77-96, device branch)
    got = torch_ops.fused_leaky_relu(x, b, 0.2, 2 ** 0.5)
    assert np.abs(got.cpu().numpy() - g["fba_out"]).max() < 1e-6
    # EqualLinear(activation) (gpen_model.py:160-162): 2-D input, bias per column
    x2 = torch.from_numpy(synth.hash_array("golden.fba.x2", (3, 16))).to(DEV)
    b2 = torch.from_numpy(synth.hash_array("golden.fba.b2", (16,))).to(DEV)
    assert np.abs(torch_ops.fused_leaky_relu(x2, b2).cpu().numpy() - g["fba2_out"]).max() < 1e-6
    # the raw op with the FusedLeakyReLUFunction.forward arguments (fused_act.py:60-61)
    raw = torch_ops.fused.fused_bias_act(x, b, x.new_empty(0), 3, 0, 0.2, 2 ** 0.5)
    assert torch.equal(raw, got)
    xi = torch.from_numpy(synth.hash_array("golden.ufd.x", (2, 3, 9, 11))).to(DEV)
    forms = {"up2": (2, 1, (2, 1)),        # Upsample (gpen_model.py:54)
             "down2": (1, 2, (1, 1)),      # Downsample (:76)
             "blur22": (1, 1, (2, 2)),     # Blur before the stride-2 encoder convs (:96, :572-581)
             "blur11": (1, 1, (1, 1))}     # Blur after the transposed modulated conv (:257-268)
    for name, (up, down, pad) in forms.items():
        out = torch_ops.upfirdn2d(xi, _blur_kernel(up), up=up, down=down, pad=pad)
        exp = g[f"ufd_{name}"]
        assert out.shape == exp.shape, (name, out.shape, exp.shape)
        assert np.abs(out.cpu().numpy() - exp).max() < 1e-6, name


def test_upfirdn2d_op_minor_and_errors():
    from oracle.enhancers import upfirdn2d as ref_upfirdn2d
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 7, 9, 3, generator=g)                     # [major, H, W, minor]
    k = torch.randn(3, 4, generator=g)
    out = torch_ops.upfirdn2d_op.upfirdn2d(x.to(DEV), k.to(DEV), 2, 2, 1, 1, 2, 1, 2, 1)
    ref = ref_upfirdn2d(x.permute(0, 3, 1, 2), k, up=2, down=1, pad=(2, 1)).permute(0, 2, 3, 1)
    assert out.shape == ref.shape and (out.cpu() - ref).abs().max() < 1e-5
    with pytest.raises(RuntimeError):                            # empty output: the reference returned garbage
        torch_ops.upfirdn2d_op.upfirdn2d(x.to(DEV), torch.ones(16, 16, device=DEV), 1, 1, 1, 1, 0, 0, 0, 0)


@pytest.mark.parametrize("prec", ["f32", "f16x3"])
def test_conv2d_nhwc_op_matches_engine_path(prec):
    ctx = ops.Ctx(DEV)
    n, cin, h, w, cout = 2, 64, 14, 12, 96
    g = torch.Generator().manual_seed(5)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    bias = torch.randn(cout, generator=g)
    x = torch.randn(n, h, w, cin, generator=g).to(DEV)
    cw = ops.ConvW(wt, bias, DEV, padding=1)
    code = {"f32": ops.PREC_F32, "f16x3": ops.PREC_F16X3}[prec]
    split = cw.wt_x3(ctx, code) if code != ops.PREC_F32 else None
    y = torch_ops.load().conv2d_nhwc(x, cw.wt, split, cw.split_scale(code), cout, 3, 3, [1, 1], [1, 1], [1, 1],
                                     ops.IN_DIRECT, ops.PAD_ZERO, cw.scale, cw.shift, ops.ACT_LRELU, 0.2, None, False,
                                     code, False)
    prev = ops.set_precision(prec)
    try:
        ye = ops.NHWC.empty(n, h, w, cout, DEV)
        ops.conv2d(ctx, ops.NHWC(x), cw, ye, act=ops.ACT_LRELU, alpha=0.2)
    finally:
        ops.set_precision(prev)
    assert torch.equal(y, ye.t)
    ref = F.leaky_relu(F.conv2d(x.permute(0, 3, 1, 2).double().cpu(), wt.double(), bias.double(), padding=1), 0.2)
    assert (y.permute(0, 3, 1, 2).double().cpu() - ref).abs().max() < 1e-4
    # pooled form (ResBlock conv1 + x0.5)
    yp = torch_ops.load().conv2d_nhwc(x, cw.wt, split, cw.split_scale(code), cout, 3, 3, [1, 1], [1, 1], [1, 1],
                                      ops.IN_DIRECT, ops.PAD_ZERO, cw.scale, cw.shift, ops.ACT_LRELU, 0.2, None, False,
                                      code, True)
    assert (yp.permute(0, 3, 1, 2).double().cpu() - F.avg_pool2d(ref, 2)).abs().max() < 1e-4


def test_norm_attention_fft_resize_ops():
    s2v = torch_ops.load()
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(2, 12, 10, 40, generator=g) * 3 + 1).to(DEV)
    wgt, b = torch.randn(40, generator=g).to(DEV), torch.randn(40, generator=g).to(DEV)
    y = s2v.layernorm2d(x, wgt, b, 1e-5, ops.ACT_LRELU, 0.1, False)
    xc = x.permute(0, 3, 1, 2).double().cpu()
    ref = F.leaky_relu(F.layer_norm(xc, xc.shape[1:], wgt.double().cpu()[:, None, None].expand(xc.shape[1:]),
                                    b.double().cpu()[:, None, None].expand(xc.shape[1:]), 1e-5), 0.1)
    assert (y.permute(0, 3, 1, 2).double().cpu() - ref).abs().max() < 2e-5
    gam, bet = torch.randn(2, 40, generator=g).to(DEV), torch.randn(2, 40, generator=g).to(DEV)
    y = s2v.instnorm_adain(x, gam, bet, 1e-5, ops.ACT_LRELU, 0.01)
    ref = F.leaky_relu(F.instance_norm(xc, eps=1e-5) * (1 + gam.double().cpu()[:, :, None, None])
                       + bet.double().cpu()[:, :, None, None], 0.01)
    assert (y.permute(0, 3, 1, 2).double().cpu() - ref).abs().max() < 2e-5
    q, k, v = (torch.randn(2, 144, 256, generator=g).to(DEV) for _ in range(3))
    o = s2v.attention(q, k, v, 4, 0.125)
    qq, kk, vv = (t.double().cpu().reshape(2, 144, 4, 64).transpose(1, 2) for t in (q, k, v))
    ref = (torch.softmax(qq @ kk.transpose(-1, -2) * 0.125, -1) @ vv).transpose(1, 2).reshape(2, 144, 256)
    assert (o.double().cpu() - ref).abs().max() < 1e-5
    xf = torch.randn(2, 12, 12, 32, generator=g).to(DEV)
    tables = ops.fft_tables(12, 12, DEV)
    spec = s2v.rfft2(xf, tables)
    back = s2v.irfft2(spec, tables, 12, 12, xf)
    assert (back - 2 * xf).abs().max() < 1e-4                 # irfft2(rfft2(x)) + x
    img = torch.rand(2, 3, 384, 384, generator=g).to(DEV)
    r = s2v.resize_bilinear(img, 96, 96, 4.0, 4.0, 0)
    assert (r.cpu() - F.interpolate(img.cpu(), (96, 96), mode="bilinear", align_corners=False)).abs().max() < 2e-6


def test_flow_warp_and_mel_ops(golden):
    from oracle import audio as ref_audio
    from s2v_amd import audio
    s2v = torch_ops.load()
    gd = golden("ops")
    flow = torch.from_numpy(synth.hash_array("golden.flow", (2, 2, 16, 16), -3.0, 3.0)).to(DEV)
    src = torch.from_numpy(synth.hash_array("golden.flow.src", (2, 3, 64, 64))).to(DEV)
    assert np.abs(s2v.flow_warp(flow, src).cpu().numpy() - gd["warp"]).max() < 2e-5
    t = np.arange(16000) / 16000.0
    wav = (0.2 * np.sin(2 * np.pi * 440 * t)).astype(np.float32)
    mel = s2v.mel_spectrogram(torch.from_numpy(wav).to(DEV), audio.tables(torch.device(DEV)), False)
    assert np.abs(mel.cpu().numpy() - ref_audio.melspectrogram(wav)).max() < 1e-3


@pytest.mark.parametrize("up,down,pad", [(1, 1, (2, 1)), (1, 1, (1, 1)), (2, 1, (2, 1)), (1, 2, (1, 1)),
                                         (1, 2, (2, 2)), (2, 1, (1, 2))])
def test_upfirdn2d_plane_tiles_ragged(up, down, pad):
    """The LDS-tiled plane kernel (NCHW inputs, 4x4 filter, 16 x 64 output tiles): sizes that leave
    partial tiles in both directions, asymmetric pads, against the reference's CPU upfirdn2d."""
    from oracle.enhancers import upfirdn2d as ref_upfirdn2d
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 5, 37, 150, generator=g)
    k = torch.randn(4, 4, generator=g)
    got = torch_ops.upfirdn2d(x.to(DEV), k.to(DEV), up=up, down=down, pad=pad)
    ref = ref_upfirdn2d(x, k, up=up, down=down, pad=pad)
    assert got.shape == ref.shape
    assert (got.cpu() - ref).abs().max() < 1e-5


def test_fused_bias_act_row_form():
    """The float4 row kernel (step_b % 4 == 0: every [N, C, H, W] activation of GPEN) in all the
    act / grad modes the reference's kernel implements (fused_bias_act_kernel.cu:36-45)."""
    g = torch.Generator().manual_seed(13)
    x = torch.randn(2, 8, 8, 12, generator=g)
    b = torch.randn(8, generator=g)
    ref_in = torch.randn(2, 8, 8, 12, generator=g)
    op = torch_ops.fused.fused_bias_act
    xb = x + b[None, :, None, None]
    exp = {(3, 0): torch.where(xb > 0, xb, xb * 0.2) * 1.5, (3, 1): torch.where(ref_in > 0, xb, xb * 0.2) * 1.5,
           (1, 0): xb * 1.5}
    for (act, grad), e in exp.items():
        got = op(x.to(DEV), b.to(DEV), ref_in.to(DEV) if grad else x.new_empty(0).to(DEV), act, grad, 0.2, 1.5)
        assert (got.cpu() - e).abs().max() < 1e-6, (act, grad)
    got = torch_ops.fused_leaky_relu(x.to(DEV), b.to(DEV), 0.2, 2 ** 0.5)
    assert (got.cpu() - torch.where(xb > 0, xb, xb * 0.2) * 2 ** 0.5).abs().max() < 1e-5


def _f16_bound(exact):
    """Stated float16 tolerance: the drop-in computes in fp32 and rounds once, so it lies within half
    an f16 ulp (<= 2^-11 |v|) of the exact result; allow 2^-10 |v| plus the subnormal spacing 2^-24."""
    return 2.0 ** -10 * np.abs(exact) + 2.0 ** -24


@pytest.mark.parametrize("dtype", [torch.float64, torch.float16])
def test_gpen_ops_half_and_double_match_reference_fallbacks(golden, dtype):
    """The dtypes the reference dispatches (AT_DISPATCH_FLOATING_TYPES_AND_HALF:
    fused_bias_act_kernel.cu:79, upfirdn2d_kernel.cu:225) through torch.ops.s2v, against the
    reference's CPU fallbacks run in that dtype (tests/golden/make_golden.py gen_ops).
    Tolerances: float64 1e-12 absolute (values are O(1)); float16 within one f16 ulp of the exact
    (fp64) result on the half-rounded inputs, and within two ulps of the fallback's own half output
    (it rounds after every torch op)."""
    g = golden("ops")
    tag = "f64" if dtype == torch.float64 else "f16"
    x = torch.from_numpy(synth.hash_array("golden.fba.x", (2, 8, 5, 7))).to(DEV, dtype)
    b = torch.from_numpy(synth.hash_array("golden.fba.b", (8,))).to(DEV, dtype)
    outs = {"fba": torch_ops.fused_leaky_relu(x, b, 0.2, 2 ** 0.5)}
    raw = torch_ops.fused.fused_bias_act(x, b, x.new_empty(0), 3, 0, 0.2, 2 ** 0.5)
    assert raw.dtype == dtype and torch.equal(raw, outs["fba"])
    xi = torch.from_numpy(synth.hash_array("golden.ufd.x", (2, 3, 9, 11))).to(DEV, dtype)
    for name, (up, down, pad) in {"up2": (2, 1, (2, 1)), "blur22": (1, 1, (2, 2)), "down2": (1, 2, (1, 1))}.items():
        outs[f"ufd_{name}"] = torch_ops.upfirdn2d(xi, _blur_kernel(up).to(dtype), up=up, down=down, pad=pad)
    for key, got in outs.items():
        assert got.dtype == dtype, key
        got = got.cpu().double().numpy()
        ref_key = f"fba_{tag}_out" if key == "fba" else f"{key}_{tag}"
        ref = g[ref_key].astype(np.float64)
        assert got.shape == ref.shape, key
        if dtype == torch.float64:
            assert np.abs(got - ref).max() < 1e-12, key
        else:
            exact = g["fba_f16_exact" if key == "fba" else f"{key}_f16_exact"]
            assert (np.abs(got - exact) <= _f16_bound(exact)).all(), (key, np.abs(got - exact).max())
            assert (np.abs(got - ref) <= 2 * _f16_bound(ref)).all(), (key, np.abs(got - ref).max())


def test_gpen_ops_dtype_rules():
    """float16 / float64 go through the row kernel (step_b % 4 == 0) and the generic kernels too;
    a dtype the reference does not dispatch, or a kernel / bias of another dtype, raises."""
    gen = torch.Generator().manual_seed(17)
    for dt in (torch.float16, torch.float64):
        x = torch.randn(2, 8, 8, 12, generator=gen).to(dt)
        b = torch.randn(8, generator=gen).to(dt)
        r = torch.randn(2, 8, 8, 12, generator=gen).to(dt)
        xb = x.double() + b.double()[None, :, None, None]
        for (act, grad), e in {(3, 0): torch.where(xb > 0, xb, xb * 0.2) * 1.5,
                               (3, 1): torch.where(r.double() > 0, xb, xb * 0.2) * 1.5, (1, 0): xb * 1.5}.items():
            got = torch_ops.fused.fused_bias_act(x.to(DEV), b.to(DEV), r.to(DEV) if grad else x.new_empty(0).to(DEV),
                                                  act, grad, 0.2, 1.5).cpu().double()
            tol = 1e-12 if dt == torch.float64 else torch.from_numpy(_f16_bound(e.numpy()))
            assert ((got - e).abs() <= tol).all(), (dt, act, grad)
        x5 = torch.randn(3, 5, 7, generator=gen).to(dt)                     # step_b = 7: element kernel
        b5 = torch.randn(5, generator=gen).to(dt)
        e5 = x5.double() + b5.double()[None, :, None]
        e5 = torch.where(e5 > 0, e5, e5 * 0.2) * 2 ** 0.5
        got5 = torch_ops.fused_leaky_relu(x5.to(DEV), b5.to(DEV)).cpu().double()
        assert ((got5 - e5).abs() <= (1e-12 if dt == torch.float64 else torch.from_numpy(_f16_bound(e5.numpy())))).all()
        xm = torch.randn(2, 7, 9, 3, generator=gen).to(dt)                  # minor > 1, 3x4 kernel: generic kernel
        km = torch.randn(3, 4, generator=gen).to(dt)
        from oracle.enhancers import upfirdn2d as ref_upfirdn2d
        em = ref_upfirdn2d(xm.double().permute(0, 3, 1, 2), km.double(), up=2, down=1, pad=(2, 1)).permute(0, 2, 3, 1)
        gm = torch_ops.upfirdn2d_op.upfirdn2d(xm.to(DEV), km.to(DEV), 2, 2, 1, 1, 2, 1, 2, 1).cpu().double()
        assert gm.shape == em.shape
        # fp32 accumulation of up to 12 half products before the single rounding
        tol = 1e-12 if dt == torch.float64 else torch.from_numpy(_f16_bound(em.numpy())) + 1e-5
        assert ((gm - em).abs() <= tol).all(), dt
    with pytest.raises(RuntimeError):
        torch_ops.fused.fused_bias_act(torch.ones(4, 4, dtype=torch.bfloat16, device=DEV),
                                       torch.ones(4, dtype=torch.bfloat16, device=DEV), torch.empty(0, device=DEV),
                                       3, 0, 0.2, 1.0)
    with pytest.raises(RuntimeError):
        torch_ops.fused.fused_bias_act(torch.ones(4, 4, dtype=torch.float16, device=DEV),
                                       torch.ones(4, device=DEV), torch.empty(0, device=DEV), 3, 0, 0.2, 1.0)
    with pytest.raises(RuntimeError):
        torch_ops.upfirdn2d_op.upfirdn2d(torch.ones(1, 8, 8, 1, dtype=torch.float64, device=DEV),
                                         torch.ones(4, 4, device=DEV), 1, 1, 1, 1, 1, 1, 1, 1)


class _NoLaunchLib:
    """libs2v ctypes handle that refuses every kernel launch (host-only queries pass through)."""
    HOST = {"s2v_conv2d_plan", "s2v_conv2d_ws_bytes", "s2v_tune", "s2v_last_error", "s2v_device_cus", "s2v_version",
            "s2v_layernorm2d_ws_bytes", "s2v_instnorm_ws_bytes", "s2v_fft_tables_floats"}

    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        if name.startswith("s2v_") and name not in self.HOST:
            raise AssertionError(f"{name} launched through ctypes on the model path")
        return getattr(self._lib, name)


@pytest.mark.parametrize("model", ["enet", "dnet"])
def test_model_forward_dispatches_through_torch_ops(model, monkeypatch):
    """the model forwards reach the kernels through the ``torch.ops.s2v``
    dispatcher (inference.py:266 / facing.py:189 call sites): a torch.profiler trace shows the
    s2v:: launch ops, and no kernel is launched through ctypes."""
    from torch.profiler import ProfilerActivity, profile
    from s2v_amd import _lib, models
    from helpers import synth_sd
    monkeypatch.setattr(_lib, "_lib", _NoLaunchLib(_lib.load()))
    if model == "enet":
        m = models.ENet()
        m.load_state_dict(synth_sd("enet"))
        args = [torch.from_numpy(a).to(DEV) for a in synth.lipsync_inputs("dispatch", 2, 256)]
    else:
        m = models.DNet()
        m.load_state_dict(synth_sd("dnet"))
        args = [torch.from_numpy(a).to(DEV) for a in synth.dnet_inputs("dispatch", 1, 256)]
    m.eval()
    m(*args)                                          # builds the engine (weight folding / splits) first
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        m(*args)
        torch.cuda.synchronize()
    names = {}
    for ev in prof.events():
        if ev.name.startswith("s2v::"):
            names[ev.name] = names.get(ev.name, 0) + 1
    convs = names.get("s2v::conv2d_", 0) + names.get("s2v::modulated_conv2d_", 0)
    assert convs > (100 if model == "enet" else 40), names
    assert names.get("s2v::instnorm_", 0) > 0 and names.get("s2v::resize_", 0) > 0, names
