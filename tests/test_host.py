"""CPU tests: the C ABI library loads and exports what include/s2v.h declares, struct layout,
state_dict layout vs the reference manifests, weight packing / folding, DFT matrices, mel host
logic and the mel restatement cross-checks.  No GPU compute here."""
import ctypes
import json
import os
import re
import shutil
import subprocess

import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from conftest import GOLDEN, REPO
from helpers import GFPGAN_KW
from s2v_amd import _lib, synth
from s2v_amd.models import arch

HEADER = os.path.join(REPO, "include", "s2v.h")


def _ea():
    from s2v_amd.models import enhancer_arch
    return enhancer_arch


def _pa():
    from s2v_amd.models import parse_arch
    return parse_arch


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(s2v_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"libs2v.so does not export {n}"
    assert set(names) == set(_lib.EXPORTS), (set(names) ^ set(_lib.EXPORTS))
    assert lib.s2v_version().startswith(b"s2v")


def test_invalid_arguments_are_rejected_without_a_device():
    lib = _lib.load()
    p = _lib.ConvParams()                       # null pointers
    assert lib.s2v_conv2d(ctypes.byref(p), None) == -1
    assert b"null" in lib.s2v_last_error()
    assert lib.s2v_upfirdn2d(None, 1, 4, 4, 1, None, 4, 4, 1, 1, 1, 1, 0, 0, 0, 0, None, 1, 1, None) == -1


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_conv_params_struct_layout_matches_header(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "%s"\n'
                   'int main(){printf("%%zu %%zu %%zu %%zu %%zu %%zu %%zu\\n", sizeof(s2v_conv_params),'
                   'offsetof(s2v_conv_params, ws), offsetof(s2v_conv_params, x_bs),'
                   'offsetof(s2v_conv_params, res), offsetof(s2v_conv_params, force_splits),'
                   'offsetof(s2v_conv_params, b_kn), offsetof(s2v_conv_params, wt_scale));return 0;}' % HEADER)
    exe = tmp_path / "sz"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    P = _lib.ConvParams
    assert got == [ctypes.sizeof(P), P.ws.offset, P.x_bs.offset, P.res.offset, P.force_splits.offset, P.b_kn.offset,
                   P.wt_scale.offset]


@pytest.mark.parametrize("name,ctor", [("lnet", lambda: arch.LNetParams()),
                                       ("enet", lambda: arch.ENetParams(lnet=arch.LNetParams())),
                                       ("dnet", lambda: arch.DNetParams()),
                                       ("gfpgan", lambda: _ea().GFPGANv1CleanParams(**GFPGAN_KW)),
                                       ("gpen", lambda: _ea().FullGeneratorParams(512, 512, 8, 2)),
                                       ("parsenet", lambda: _pa().ParseNetParams(**_pa().face_parse_net(512)))])
def test_state_dict_layout_matches_reference(name, ctor):
    ref = json.load(open(os.path.join(GOLDEN, f"{name}_keys.json")))
    mine = {k: list(v.shape) for k, v in ctor().state_dict().items()}
    assert mine == ref


def test_public_models_share_the_layout():
    from s2v_amd import models
    assert set(models.ENet().state_dict()) == set(json.load(open(os.path.join(GOLDEN, "enet_keys.json"))))
    assert set(models.DNet().state_dict()) == set(json.load(open(os.path.join(GOLDEN, "dnet_keys.json"))))


def test_synth_is_deterministic_and_portable():
    u = synth.hash_uniform("decoder.res2.res0.conv1.ffc.convl2l.weight", 4)
    # fixed values: the golden fixtures were produced from exactly these numbers
    np.testing.assert_allclose(u, synth.hash_uniform("decoder.res2.res0.conv1.ffc.convl2l.weight", 4))
    assert np.all(np.abs(u) < 1)
    a = synth.synth_tensor("x.running_var", (5,))
    assert np.all(a > 0.7)
    assert synth.synth_tensor("style_convs.0.weight", (1,))[0] == 0.0


def test_conv_weight_packing_roundtrip():
    from s2v_amd.ops import ConvW
    w = torch.randn(5, 7, 3, 3)
    cw = ConvW(w, torch.randn(5), "cpu", padding=1)
    assert cw.kpad % 32 == 0 and cw.npad % 128 == 0
    back = cw.wt[:5, :63].reshape(5, 3, 3, 7).permute(0, 3, 1, 2)
    assert torch.equal(back, w)
    assert torch.all(cw.wt[5:] == 0) and torch.all(cw.wt[:, 63:] == 0)
    wt = torch.randn(7, 5, 3, 3)                        # ConvTranspose2d layout [in, out, k, k]
    ct = ConvW(wt, None, "cpu", transposed=True, stride=2, padding=1, output_padding=1)
    assert (ct.cout, ct.cin) == (5, 7) and ct.out_hw(6, 6) == (12, 12)
    c1 = ConvW(torch.randn(4, 3, 3), None, "cpu", dilation=(1, 3))   # Conv1d k3 dil3 (DNet.py:41-42)
    assert (c1.kh, c1.kw, c1.dw) == (1, 3, 3) and c1.out_hw(1, 20) == (1, 14)


def test_bn_fold_matches_eval_batchnorm():
    from s2v_amd.ops import ConvW
    g = torch.Generator().manual_seed(0)
    w, b = torch.randn(6, 4, 3, 3, generator=g), torch.randn(6, generator=g)
    bn = (torch.rand(6, generator=g) + 0.5, torch.randn(6, generator=g), torch.randn(6, generator=g),
          torch.rand(6, generator=g) + 0.5)
    cw = ConvW(w, b, "cpu", padding=1, bn=bn)
    x = torch.randn(2, 4, 5, 5, generator=g)
    ref = torch.nn.functional.batch_norm(torch.nn.functional.conv2d(x, w, b, padding=1), bn[2], bn[3], bn[0], bn[1],
                                         False, 0.0, 1e-5)
    got = torch.nn.functional.conv2d(x, w, None, padding=1) * cw.scale[None, :, None, None] + cw.shift[None, :, None, None]
    assert (got - ref).abs().max() < 1e-5


def test_spectral_norm_fold_matches_torch():
    from s2v_amd.engine.common import conv_weight
    from torch.nn.utils import spectral_norm
    m = spectral_norm(torch.nn.Conv2d(4, 6, 3))
    sd = synth.synth_torch_state_dict(m)
    m.load_state_dict(sd)
    m.eval()
    with torch.no_grad():
        m(torch.zeros(1, 4, 5, 5))          # the spectral-norm pre-hook recomputes .weight
    assert (conv_weight(sd, "") - m.weight).abs().max() < 1e-6


def test_fourier_matrices_are_the_reference_transforms():
    from s2v_amd.ops import fourier_matrices
    for h, w in ((12, 12), (24, 24), (6, 10)):
        d2, iv = fourier_matrices(h, w, "cpu")
        x = torch.randn(3, h, w, dtype=torch.float64)
        spec = torch.fft.rfftn(x, dim=(-2, -1), norm="ortho")
        st = torch.stack([spec.real, spec.imag], -1).reshape(3, -1)
        assert (d2.double() @ x.reshape(3, -1).t()).t().sub(st).abs().max() < 1e-5
        y = torch.randn_like(st)          # arbitrary spectrum, incl. imag DC / Nyquist parts
        ref = torch.fft.irfftn(torch.complex(y[:, 0::2], y[:, 1::2]).reshape(3, h, w // 2 + 1), s=(h, w),
                               dim=(-2, -1), norm="ortho").reshape(3, -1)
        assert (iv.double() @ y.t()).t().sub(ref).abs().max() < 1e-5


def test_adain_bank_layout():
    from s2v_amd.engine.common import AdainBank
    sd = {}
    for p, c in (("a.", 3), ("b.", 5)):
        sd.update({p + "mlp_shared.0.weight": torch.randn(128, 7), p + "mlp_shared.0.bias": torch.randn(128),
                   p + "mlp_gamma.weight": torch.randn(c, 128), p + "mlp_gamma.bias": torch.randn(c),
                   p + "mlp_beta.weight": torch.randn(c, 128), p + "mlp_beta.bias": torch.randn(c)})
    bank = AdainBank(7)
    gid = bank.add_group(sd, [("a.", 3), ("b.", 5)])
    bank.build("cpu")
    assert bank.total == 16 and bank.groups[gid] == (0, 8)
    assert bank.seg.tolist() == [0] * 3 + [1] * 5 + [0] * 3 + [1] * 5
    assert torch.equal(bank.w2t[:, 3:8].t(), sd["b.mlp_gamma.weight"])
    assert torch.equal(bank.w2t[:, 11:16].t(), sd["b.mlp_beta.weight"])


def test_mel_chunk_starts_follow_inference_loop():
    from s2v_amd.audio import chunk_starts
    from oracle.audio import mel_chunk_starts
    for T in (16, 17, 100, 3201):
        assert chunk_starts(T) == mel_chunk_starts(T)
    st = chunk_starts(3201)
    assert st[:4] == [0, 3, 6, 9] and st[-1] == 3201 - 16
    assert len(st) == 997           # 40 s at 16 kHz: the last window is clamped (inference.py:212-214)


def test_mel_restatement_cross_checks():
    """The NumPy restatement against independent implementations: scipy's lfilter for the
    pre-emphasis and torch.stft for the framed, windowed STFT."""
    from scipy import signal
    from oracle import audio
    from s2v_amd.audio import slaney_mel_basis
    rng = np.random.default_rng(0)
    wav = (0.1 * rng.standard_normal(16000)).astype(np.float32)
    assert np.abs(audio.preemphasis(wav) - signal.lfilter([1, -0.97], [1], wav)).max() < 1e-12
    y = audio.preemphasis(wav)
    for mode in ("constant", "reflect"):
        ref = torch.stft(torch.from_numpy(y), 800, 200, 800, torch.hann_window(800, periodic=True, dtype=torch.float64),
                         center=True, pad_mode=mode, return_complex=True).abs().numpy()
        assert np.abs(audio.stft_mag(y, mode) - ref).max() < 1e-9
    mel = audio.melspectrogram(wav)
    assert mel.shape == (80, 81) and mel.min() >= -4 and mel.max() <= 4
    b = audio.mel_basis()
    assert b.shape == (80, 401) and b.dtype == np.float32
    assert np.array_equal(b, slaney_mel_basis())


def test_gpen_synthetic_blur_kernels_are_the_fixed_buffers():
    from helpers import synth_sd
    sd = synth_sd("gpen")
    k = torch.tensor([1.0, 3.0, 3.0, 1.0])
    k = k[None, :] * k[:, None] / 64.0
    assert torch.equal(sd["ecd1.0.0.kernel"], k)
    assert torch.equal(sd["generator.convs.0.conv.blur.kernel"], 4 * k)
    assert torch.equal(sd["generator.to_rgbs.0.upsample.kernel"], 4 * k)
    assert float(sd["generator.conv1.noise.weight"]) == pytest.approx(0.1)


def test_fft_tables_reproduce_torch_fft():
    """The separable passes s2v_rfft2 / s2v_irfft2 run, emulated with the host-built tables."""
    from s2v_amd.ops import fft_tables
    for h, w in ((12, 12), (24, 24), (48, 48), (6, 10)):
        wf = w // 2 + 1
        t = fft_tables(h, w, "cpu").double()
        o = 0
        fw = t[o:o + 2 * wf * w].reshape(w, 2, wf).permute(1, 2, 0); o += 2 * wf * w     # -> [2, v, w]
        fh = t[o:o + 2 * h * h].reshape(h, 2, h).permute(1, 2, 0); o += 2 * h * h        # -> [2, u, h]
        ih = t[o:o + 2 * h * h].reshape(h, 2, h).permute(1, 2, 0); o += 2 * h * h        # -> [2, h, u]
        iw = t[o:].reshape(wf, 2, w).permute(1, 2, 0)                                     # -> [2, w, v]
        x = torch.randn(3, h, w, dtype=torch.float64)
        yr, yi = x @ fw[0].t(), x @ fw[1].t()                              # W pass: [c, h, v]
        zr = fh[0] @ yr - fh[1] @ yi                                       # H pass (complex)
        zi = fh[1] @ yr + fh[0] @ yi
        ref = torch.fft.rfftn(x, dim=(-2, -1), norm="ortho")
        assert (zr - ref.real).abs().max() < 1e-5 and (zi - ref.imag).abs().max() < 1e-5
        sr, si = torch.randn(3, h, wf, dtype=torch.float64), torch.randn(3, h, wf, dtype=torch.float64)
        ar = ih[0] @ sr - ih[1] @ si                                       # inverse H pass
        ai = ih[1] @ sr + ih[0] @ si
        y = ar @ iw[0].t() + ai @ iw[1].t()                                # c2r W pass
        ref = torch.fft.irfftn(torch.complex(sr, si), s=(h, w), dim=(-2, -1), norm="ortho")
        assert (y - ref).abs().max() < 1e-5


def test_rrdb_unshuffle_fold_equals_pixel_unshuffle_conv():
    """engine/rrdb.py folds pixel_unshuffle(x, r) + 3x3 conv (rrdbnet_arch.py:105-110) into one
    (3r)x(3r) stride-r pad-r conv of the image; check the weight permutation on CPU for r = 2, 4."""
    import torch
    import torch.nn.functional as F
    from oracle.sr import pixel_unshuffle
    from s2v_amd.engine.rrdb import _unshuffle_weight
    g = torch.Generator().manual_seed(0)
    for r in (2, 4):
        x = torch.randn(2, 3, 8 * r, 4 * r, generator=g, dtype=torch.float64)
        w = torch.randn(5, 3 * r * r, 3, 3, generator=g, dtype=torch.float64)
        ref = F.conv2d(pixel_unshuffle(x, r), w, None, 1, 1)
        got = F.conv2d(x, _unshuffle_weight(w, r, 3), None, r, r)
        assert got.shape == ref.shape and torch.allclose(got, ref, atol=1e-10), r


def test_rrdb_gflop_matches_flop_counter():
    """models.sr_arch.rrdb_gflop (the sr bench's GFLOP per frame) == torch's FlopCounterMode on the
    oracle forward, for every scale."""
    import torch
    from torch.utils.flop_counter import FlopCounterMode
    from oracle.sr import rrdbnet_forward
    from s2v_amd.models.sr_arch import RRDBNetParams, rrdb_gflop
    for scale in (1, 2, 4):
        sd = {k: v.float() for k, v in RRDBNetParams(3, 3, scale=scale, num_feat=32, num_block=2).state_dict().items()}
        x = torch.zeros(1, 3, 16, 12)
        with FlopCounterMode(display=False) as fc, torch.no_grad():
            rrdbnet_forward(sd, x, scale)
        assert abs(fc.get_total_flops() / 1e9 - rrdb_gflop(16, 12, scale, num_block=2)) < 1e-9, scale


def test_torch_custom_ops_registered_hip_only():
    """TORCH_LIBRARY(s2v) (csrc/torch_ops.cpp): every op is registered with the reference's schema for
    the GPEN drop-ins, and a CPU tensor raises (no CPU kernel, no fallback)."""
    from s2v_amd import torch_ops
    ns = torch_ops.load()
    for name in torch_ops.OPS + torch_ops.LAUNCH_OPS:
        assert hasattr(ns, name), name
    for name in torch_ops.LAUNCH_OPS:           # launch ops mutate caller-owned outputs
        assert "(a!)" in str(getattr(ns, name).default._schema), name
    with pytest.raises(NotImplementedError):
        ns.fill_value_(torch.zeros(4), 1.0)
    assert str(ns.fused_bias_act.default._schema) == (
        "s2v::fused_bias_act(Tensor input, Tensor bias, Tensor refer, int act, int grad, float alpha, "
        "float scale) -> Tensor")
    assert str(ns.upfirdn2d.default._schema) == (
        "s2v::upfirdn2d(Tensor input, Tensor kernel, int up_x, int up_y, int down_x, int down_y, int pad_x0, "
        "int pad_x1, int pad_y0, int pad_y1) -> Tensor")
    with pytest.raises(NotImplementedError):
        torch_ops.fused.fused_bias_act(torch.zeros(2, 3), torch.zeros(3), torch.zeros(0), 3, 0, 0.2, 1.0)
    with pytest.raises(NotImplementedError):
        torch_ops.upfirdn2d(torch.zeros(1, 2, 4, 4), torch.ones(2, 2))


def _plan(n, h, w, cin, cout, k=3, stride=1, pad=1, force_tile=0, in_scale=False, batch=0):
    """s2v_conv2d_plan of an f16x3 direct conv (host-only: fake aligned pointers, nothing launched)."""
    lib = _lib.load()
    p = _lib.ConvParams()
    p.x, p.y, p.wt_x3, p.wt = 1 << 20, 2 << 20, 3 << 20, 4 << 20
    p.n, p.h, p.w, p.cin, p.xcs = n, h, w, cin, cin
    p.kh = p.kw = k
    p.sh = p.sw = stride
    p.ph = p.pw = pad
    p.dh = p.dw = 1
    p.oh, p.ow = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    p.cout, p.ycs = cout, cout
    p.kpad = (k * k * cin + 31) // 32 * 32
    p.npad = (cout + 127) // 128 * 128 if cout <= 128 else (cout + 255) // 256 * 256
    p.prec = 2                                  # S2V_PREC_F16X3
    p.force_tile = force_tile
    if batch:                                   # per-sample weights (modulated convs): n images per member
        p.batch, p.x_bs, p.y_bs, p.w_bs = batch, n * h * w * cin, n * p.oh * p.ow * cout, p.npad * p.kpad
    if in_scale:
        p.in_scale, p.in_scale_ns = 5 << 20, cin
    out = (ctypes.c_int * 11)()
    rc = lib.s2v_conv2d_plan(ctypes.byref(p), out)
    return rc, list(out)


def test_planner_gives_narrow_3x3_layers_to_the_halo_kernel():
    """conv.hip make_plan_x3 (no GPU needed): 3x3 stride-1 layers of <= 64 / <= 128 output channels over
    a patch grid that is >= 85 % image and a chip-filling grid take conv_x3_halo<ELT, 4, 1> / <ELT, 4, 2>
    (plan A mode 8); emptier patch grids, wide layers, strided convs and small grids keep the
    implicit-GEMM tiles; forcing the halo tile where it cannot run is an error."""
    from s2v_amd import ops
    rc, pl = _plan(4, 512, 512, 128, 64, in_scale=True)
    assert rc == 0 and pl[3] == 8 and (pl[0], pl[1]) == (256, 64), pl
    assert ops.plan_symbol(pl) == "void s2v::conv_x3_halo<1, 4, 1>(s2v::ConvArgs)"
    rc, pl = _plan(4, 256, 256, 128, 128)
    assert rc == 0 and pl[3] == 8 and (pl[0], pl[1]) == (256, 128), pl
    assert ops.plan_symbol(pl) == "void s2v::conv_x3_halo<1, 4, 2>(s2v::ConvArgs)"
    for args in ((4, 200, 200, 64, 64), (16, 256, 256, 256, 256), (1, 64, 64, 64, 64), (4, 512, 512, 64, 32),
                 (16, 400, 400, 128, 128)):
        rc, pl = _plan(*args)
        assert rc == 0 and pl[3] != 8, (args, pl)
    rc, pl = _plan(4, 256, 256, 64, 64, stride=2)
    assert rc == 0 and pl[3] != 8
    rc, pl = _plan(1, 400, 400, 128, 128, batch=16)     # ENet's 400^2 StyleConv (per-sample weights): 512x128
    assert rc == 0 and pl[3] != 8, pl
    rc, pl = _plan(4, 200, 192, 64, 64)                 # ragged rows, 97 % of the patch grid: halo
    assert rc == 0 and pl[3] == 8, pl
    rc, _ = _plan(4, 256, 256, 64, 64, stride=2, force_tile=18)
    assert rc != 0 and b"conv_x3_halo" in _lib.load().s2v_last_error()
