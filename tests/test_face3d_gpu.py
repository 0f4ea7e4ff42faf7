"""3DMM extraction on the device (facing.py:100-130) against the reference goldens
(tests/golden/face3d_goldens.npz) and the CPU restatement (oracle/face3d.py, pinned in
test_face3d_host.py).

Bars:
* s2v_pil_resize_crop (Pillow's fixed-point bicubic / bilinear + crop): BIT-EXACT uint8 pixels
  (the fp32 output is pixel / 255. rounded once, compared exactly as well);
* ReconNetWrapper('resnet50') coefficients: within 1e-3 of the output scale of the fp32 reference
  in every conv arithmetic mode (53 convolutions, as the RetinaFace-R50 bar);
* the semantic rows of face_3dmm_extraction: trans_params columns EXACT (host float64 -> float32),
  coefficient columns as above.
"""
import os

import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import FACE3D_LM3D, PIL_RESIZE_CASES, face3d_frames, face3d_landmarks, synth_sd
from oracle import face3d as O3

pytestmark = pytest.mark.gpu
DEV = "cuda"
HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "face3d_goldens.npz"))
N_CASES = len(face3d_landmarks())


def _u8(x):
    """fp32 pixel / 255. back to the uint8 pixel, asserting the value is exactly float32(p / 255.)."""
    p = np.rint(x.astype(np.float64) * 255.0).astype(np.int64)
    assert np.array_equal((p / 255.).astype(np.float32), x), "not an exact pixel / 255. value"
    return p.astype(np.uint8)


def test_pil_resize_matches_pillow_goldens():
    from s2v_amd import face3d, ops
    from s2v_amd.ops import NHWC
    ctx = ops.Ctx(DEV)
    from s2v_amd import synth
    for i, (w0, h0, w, h, flt) in enumerate(PIL_RESIZE_CASES):
        img = np.floor(synth.hash_array(f"golden.pil.{i}", (h0, w0, 3), 0.0, 256.0)).astype(np.uint8)
        out = NHWC.empty(1, h, w, 4, DEV)
        face3d.resize_crop(ctx, torch.from_numpy(img).to(DEV)[None].contiguous(), [(w, h, 0, 0)], out, filter=flt)
        got = out.t[0].cpu().numpy()
        assert np.array_equal(_u8(got[..., :3]), G[f"pil_{i}"]), i
        assert (got[..., 3] == 0).all()


def test_resize_crop_batch_matches_reference_align_img():
    """All landmark cases in ONE launch (per-frame boxes, negative offsets, zero fill, ~7x downscale)."""
    from s2v_amd import face3d, ops
    from s2v_amd.ops import NHWC
    frames = face3d_frames(N_CASES)
    boxes = [tuple(int(v) for v in G[f"box_{i}"]) for i in range(N_CASES)]
    out = NHWC.empty(N_CASES, 224, 224, 4, DEV)
    face3d.resize_crop(ops.Ctx(DEV), torch.from_numpy(frames).to(DEV), boxes, out)
    got = out.t.cpu().numpy()
    for i in range(N_CASES):
        assert np.array_equal(_u8(got[i, ..., :3]), G[f"im_{i}"]), i
        assert np.array_equal(_u8(got[i, ..., :3]), O3.pil_resize_crop(frames[i], boxes[i]))


def test_align_img_drop_in():
    from s2v_amd import face3d
    frames = face3d_frames(N_CASES)
    lm = face3d.frame_landmarks(face3d_landmarks()[3], 240, 180, FACE3D_LM3D)
    trans, im, lm_new, mask = face3d.align_img(torch.from_numpy(frames[3]).to(DEV), lm, FACE3D_LM3D)
    assert mask is None and im.shape == (224, 224, 3)
    assert np.array_equal(_u8(im.cpu().numpy()), G["im_3"])
    assert np.array_equal(trans.astype(np.float32), G["semantic"][3, 257:])
    with pytest.raises(RuntimeError):
        face3d.align_img(torch.from_numpy(frames[3]), lm, FACE3D_LM3D)


@pytest.fixture(scope="module")
def recon():
    from s2v_amd import models
    m = models.define_net_recon("resnet50", use_last_fc=False, init_path="")
    m.load_state_dict(synth_sd("recon"), strict=True)
    return m.eval()


def _coeff_err(got, ref):
    return np.abs(got - ref).max() / max(1.0, np.abs(ref).max())


def test_recon_forward_matches_reference(recon, prec):
    x = torch.stack([torch.tensor(G[f"im_{i}"] / 255., dtype=torch.float32).permute(2, 0, 1) for i in range(3)])
    got = recon(x.to(DEV)).cpu().numpy()
    assert got.shape == (3, 257)
    assert _coeff_err(got, G["semantic"][:3, :257]) <= 1e-3, prec


def test_face_3dmm_extraction_matches_reference(recon, prec):
    from s2v_amd import face3d
    frames = torch.from_numpy(face3d_frames(N_CASES)).to(DEV)
    lms = face3d_landmarks()
    ext = face3d.Face3DExtractor(recon, FACE3D_LM3D, DEV, batch=4)          # ragged last batch (4 + 2)
    sem = ext.face_3dmm_extraction(frames, lms)
    assert sem.shape == (N_CASES, 262) and sem.dtype == np.float32
    assert np.array_equal(sem[:, 257:], G["semantic"][:, 257:])
    assert _coeff_err(sem[:, :257], G["semantic"][:, :257]) <= 1e-3, prec
    whole = face3d.Face3DExtractor(recon, FACE3D_LM3D, DEV, batch=32).face_3dmm_extraction(frames, lms)
    assert np.array_equal(whole[:, 257:], sem[:, 257:])
    assert _coeff_err(whole[:, :257], sem[:, :257]) <= 1e-5
    exp = ext.expression(frames[0], lms[0])
    assert exp.shape == (64,) and np.allclose(exp.numpy(), sem[0, 80:144], atol=1e-5)


def test_resize_crop_rejects_bad_inputs():
    from s2v_amd import face3d, ops
    from s2v_amd.ops import NHWC
    ctx = ops.Ctx(DEV)
    out = NHWC.empty(1, 8, 8, 4, DEV)
    fr = torch.zeros((1, 240, 240, 3), dtype=torch.uint8, device=DEV)
    with pytest.raises(ValueError, match="downscale"):
        face3d.resize_crop(ctx, fr, [(20, 20, 0, 0)], out)               # 12x > the 48-tap limit
    with pytest.raises(RuntimeError):
        face3d.resize_crop(ctx, fr.float(), [(100, 100, 0, 0)], out)
    lib = ctx.lib
    params = torch.tensor([[100, 100, 0, 0]], dtype=torch.int32, device=DEV)
    assert lib.s2v_pil_resize_crop(fr.data_ptr(), 1, 240, 240, 240 * 240 * 3, params.data_ptr(), 1, out.ptr, 8, 8,
                                   4, ctx.stream) != 0                    # filter 1 (NEAREST) unsupported


@pytest.mark.parametrize("box,oh,ow", [((500, 380, -20, 10), 50, 300),     # > 256 columns: row-per-block kernel
                                       ((61, 23, 3, -2), 30, 64),          # 7.8x vertical downscale: per-row fallback
                                       ((240, 180, 5, 7), 33, 200)])       # no resample at all (copy + crop)
def test_resize_crop_kernel_paths_vs_oracle(box, oh, ow):
    from s2v_amd import face3d, ops
    from s2v_amd.ops import NHWC
    frames = face3d_frames(2)
    out = NHWC.empty(2, oh, ow, 4, DEV)
    face3d.resize_crop(ops.Ctx(DEV), torch.from_numpy(frames).to(DEV), [box, box], out)
    got = out.t.cpu().numpy()
    for i in range(2):
        assert np.array_equal(_u8(got[i, ..., :3]), O3.pil_resize_crop(frames[i], box, oh, ow)), (box, i)
