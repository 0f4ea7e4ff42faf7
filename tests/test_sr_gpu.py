"""Frame super-resolution on the device (RealESRNet / RRDBNet,
third_part/GPEN/sr_model) against the goldens the reference modules produced
(tests/golden/rrdbnet_goldens.npz) and the CPU oracle (oracle/sr.py).

Tolerances.  The uint8 front / back ends (s2v_sr_u8_in, s2v_sr_f32_out) are bit-exact against the
oracle's NumPy / torch restatement.  The RRDBNet forward is fp32 over 350 convs; the synthetic
weights give outputs with |x| <= ~55, so the bounds are relative to the tensor's max magnitude:
1e-5 in f32 mode, 1e-4 in bf16x3 mode (3 * 2^-16 per product, over 69 residual blocks).
uint8 frames: never more than 1 LSB off the reference; the fraction of 1-LSB flips (values that sit
within the float error of a .5 rounding boundary) is bounded per mode.
"""
import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import RRDB_FORWARD, RRDB_PROCESS, rrdb_sd
from s2v_amd import synth

pytestmark = pytest.mark.gpu
DEV = "cuda"
FWD_REL = {"f32": 1e-5, "bf16x3": 1e-4, "f16x3": 1e-5}          # measured on MI355X: 1.4e-6 / 1.7e-5
FLIP_FRAC = {"f32": 1e-3, "bf16x3": 5e-3, "f16x3": 1e-3}        # measured: 2e-4 / 1.5e-3


def _net(scale):
    from s2v_amd import models
    m = models.RRDBNet(3, 3, scale=scale, num_feat=32, num_block=23, num_grow_ch=32)
    m.load_state_dict(rrdb_sd(scale), strict=True)
    return m.eval()


@pytest.mark.parametrize("flip", [0, 1])
def test_sr_u8_in_matches_restatement(flip):
    """s2v_sr_u8_in == real_esrnet.py:100-115 (x / 255 in fp32, BGR -> RGB, reflect pad) bit for bit."""
    from oracle import sr
    from s2v_amd import ops
    from s2v_amd.ops import NHWC
    ctx = ops.Ctx(DEV)
    img = synth.sr_frame("t.sr_in", 2, 9, 7)
    for pb, pr in ((0, 0), (1, 1), (3, 2)):
        y = NHWC.empty(2, 9 + pb, 7 + pr, 4, DEV)
        src = torch.from_numpy(img).to(DEV)
        ops.check(ctx.lib.s2v_sr_u8_in(src.data_ptr(), 2, 9, 7, flip, pb, pr, y.ptr, 4, ctx.stream), "sr_u8_in")
        for b in range(2):
            im = img[b] if flip else img[b][:, :, ::-1]
            t = torch.from_numpy(np.ascontiguousarray(im.astype(np.float32) / 255.)).permute(2, 0, 1)[[2, 1, 0]]
            ref = torch.nn.functional.pad(t[None], (0, pr, 0, pb), "reflect")[0].permute(1, 2, 0)
            got = y.t[b, :, :, :3].cpu()
            assert torch.equal(got, ref), (flip, pb, pr)
            assert (y.t[b, :, :, 3] == 0).all()
    # the oracle's own preprocessing (RGB order) agrees as well
    t, hp, wp = sr.sr_preprocess(img[0], 2)
    y = NHWC.empty(1, 10, 8, 4, DEV)
    src = torch.from_numpy(img[:1].copy()).to(DEV)
    ops.check(ctx.lib.s2v_sr_u8_in(src.data_ptr(), 1, 9, 7, 1, hp, wp, y.ptr, 4, ctx.stream), "sr_u8_in")
    assert torch.equal(y.t[0, :, :, :3].cpu(), t[0].permute(1, 2, 0))


def test_sr_u8_in_rejects_oversized_padding():
    from s2v_amd import ops, _lib
    ctx = ops.Ctx(DEV)
    x = torch.zeros((1, 2, 2, 3), dtype=torch.uint8, device=DEV)
    y = torch.empty((1, 5, 5, 4), device=DEV)
    rc = ctx.lib.s2v_sr_u8_in(x.data_ptr(), 1, 2, 2, 1, 3, 3, y.data_ptr(), 4, ctx.stream)
    assert rc != 0 and b"reflect padding" in _lib.load().s2v_last_error()


def test_sr_f32_out_matches_restatement():
    """s2v_sr_f32_out == real_esrnet.py:126-131 (crop, clamp, RGB -> BGR, NumPy round-half-even)."""
    from oracle import sr
    from s2v_amd import ops
    from s2v_amd.ops import NHWC
    ctx = ops.Ctx(DEV)
    g = torch.Generator().manual_seed(7)
    x = torch.rand((1, 3, 12, 10), generator=g) * 1.4 - 0.2
    x[0, 0, 0, :5] = torch.tensor([0.5, 1.5, 2.5, 254.5, 127.5]) / 255.0      # .5 boundaries
    ref = sr.sr_postprocess(x, 1, 2)
    xd = NHWC.empty(1, 12, 10, 3, DEV)
    ops.nchw_to_nhwc(ctx, x.to(DEV), xd)
    out = torch.empty((1, 11, 8, 3), dtype=torch.uint8, device=DEV)
    ops.check(ctx.lib.s2v_sr_f32_out(xd.ptr, 1, 11, 8, 12, 10, 3, 1, out.data_ptr(), ctx.stream), "sr_f32_out")
    assert np.array_equal(out[0].cpu().numpy(), ref)


@pytest.mark.parametrize("case", RRDB_FORWARD, ids=[c[0] for c in RRDB_FORWARD])
def test_rrdbnet_forward_matches_reference(case, prec, golden):
    tag, scale, shape = case
    ref = golden("rrdbnet_goldens")[f"fwd_{tag}"]
    x = torch.from_numpy(synth.hash_array(f"golden.rrdb.{tag}", shape, 0.0, 1.0)).to(DEV)
    y = _net(scale)(x).cpu().numpy()
    assert y.shape == ref.shape
    err = np.abs(y - ref).max() / np.abs(ref).max()
    print(f"rrdbnet {tag} {prec}: max rel err {err:.2e}")
    assert err <= FWD_REL[prec], (tag, prec, err)


@pytest.mark.parametrize("case", RRDB_PROCESS, ids=[c[0] for c in RRDB_PROCESS])
def test_realesrnet_process_matches_reference(case, prec, golden):
    """RealESRNet.process on uint8 BGR frames (odd sizes -> reflect pad; tiled variant) vs the
    reference's own uint8 output."""
    from s2v_amd.sr import RealESRNet
    tag, scale, h, w, tile, pad = case
    ref = golden("rrdbnet_goldens")[f"proc_{tag}"]
    sr = RealESRNet(scale=scale, tile_size=tile, tile_pad=pad, device=DEV, net=_net(scale))
    out = sr.process(synth.sr_frame(f"golden.rrdb.{tag}", 1, h, w)[0])
    assert out is not None and out.shape == ref.shape and out.dtype == np.uint8
    d = np.abs(out.astype(int) - ref.astype(int))
    print(f"realesrnet {tag} {prec}: max {d.max()} LSB, flips {(d > 0).mean():.4f}")
    assert d.max() <= 1 and (d > 0).mean() <= FLIP_FRAC[prec], (tag, prec, d.max(), (d > 0).mean())


def test_realesrnet_batch_matches_single_frames():
    """process_device on a batch == frame by frame (the bench path)."""
    from s2v_amd.sr import RealESRNet
    sr = RealESRNet(scale=2, device=DEV, net=_net(2))
    frames = torch.from_numpy(synth.sr_frame("t.sr_batch", 3, 20, 18)).to(DEV)
    batch = sr.process_device(frames)
    for i in range(3):
        assert torch.equal(batch[i], sr.process_device(frames[i]))


def test_realesrnet_rejects_cpu_tensors():
    from s2v_amd.sr import RealESRNet
    sr = RealESRNet(scale=2, device=DEV, net=_net(2))
    with pytest.raises(RuntimeError, match="HIP device only"):
        sr.process(torch.zeros((8, 8, 3), dtype=torch.uint8))
