"""3DMM extraction front end (preprocessing/facing.py:100-130) on the CPU: the
restatement (oracle/face3d.py) against the reference goldens (tests/golden/face3d_goldens.npz, made
by tests/golden/make_golden.py gen_face3d from the reference's preprocess.py / networks.py and from
Pillow), and the product's host glue (POS fits, landmark fix-up, split_coeff, model API layout).

Bars: Pillow resampling and the align geometry BIT-EXACT (uint8 pixels, int boxes, the float32
trans_params); the fp32 ResNet-50 restatement within 2e-5 of the reference module's output scale
(same torch CPU kernels, different op grouping).
"""
import json
import os

import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import FACE3D_CASES, FACE3D_LM3D, PIL_RESIZE_CASES, face3d_frames, face3d_landmarks, synth_sd
from oracle import face3d as O3

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "face3d_goldens.npz"))
N_CASES = len(face3d_landmarks())


@pytest.mark.parametrize("i", range(len(PIL_RESIZE_CASES)))
def test_oracle_pil_resize_matches_pillow_goldens(i):
    from s2v_amd import synth
    w0, h0, w, h, flt = PIL_RESIZE_CASES[i]
    img = np.floor(synth.hash_array(f"golden.pil.{i}", (h0, w0, 3), 0.0, 256.0)).astype(np.uint8)
    got = O3.pil_resize(img, w, h, flt)
    assert np.array_equal(got, G[f"pil_{i}"])


def test_oracle_pil_resize_matches_installed_pillow():
    """A few more shapes against Pillow itself (present in this image)."""
    Image = pytest.importorskip("PIL.Image")
    g = np.random.default_rng(1)
    for (h0, w0, h, w, flt) in ((64, 48, 23, 101, 3), (31, 77, 90, 12, 3), (50, 50, 7, 7, 3), (40, 60, 41, 59, 2)):
        img = g.integers(0, 256, (h0, w0, 3), dtype=np.uint8)
        exp = np.asarray(Image.fromarray(img).resize((w, h), resample=flt))
        assert np.array_equal(O3.pil_resize(img, w, h, flt), exp), (h0, w0, h, w, flt)


@pytest.mark.parametrize("i", range(N_CASES))
def test_oracle_align_and_crop_match_reference(i):
    frames = face3d_frames(N_CASES)
    lm = G[f"lm_{i}"]
    if FACE3D_CASES[i] is not None:          # FAN landmarks are float32 (facing.py:96); the default set is float64
        lm = lm.astype(np.float32)
    H, W = frames.shape[1:3]
    trans, box, lm_new = O3.align(W, H, lm, FACE3D_LM3D)
    gb = G[f"box_{i}"]
    assert box == (int(gb[0]), int(gb[1]), int(gb[2]), int(gb[3]))          # astype(np.int32) truncation
    assert np.array_equal(trans.astype(np.float32), G["semantic"][i, 257:])
    np.testing.assert_allclose(lm_new, G[f"lmnew_{i}"], rtol=0, atol=1e-9)
    assert np.array_equal(O3.pil_resize_crop(frames[i], box), G[f"im_{i}"])


def test_oracle_recon_forward_matches_reference():
    sd = synth_sd("recon")
    x = torch.stack([torch.tensor(G[f"im_{i}"] / 255., dtype=torch.float32).permute(2, 0, 1) for i in range(2)])
    with torch.no_grad():
        got = O3.recon_forward(sd, x).numpy()
    ref = G["semantic"][:2, :257]
    assert np.abs(got - ref).max() <= 2e-5 * max(1.0, np.abs(ref).max())


def test_product_host_glue_matches_reference():
    """s2v_amd.face3d's host-side steps (landmark fix-up, POS, box, trans_params, split_coeff)."""
    from s2v_amd import face3d
    frames = face3d_frames(N_CASES)
    H, W = frames.shape[1:3]
    for i, lm in enumerate(face3d_landmarks()):
        li = face3d.frame_landmarks(lm, W, H, FACE3D_LM3D)
        assert np.array_equal(li, G[f"lm_{i}"].astype(li.dtype))
        trans, box, lm_new = face3d.align_params(W, H, li, FACE3D_LM3D)
        gb = G[f"box_{i}"]
        assert box == (int(gb[0]), int(gb[1]), int(gb[2]), int(gb[3]))
        assert np.array_equal(trans.astype(np.float32), G["semantic"][i, 257:])
        np.testing.assert_allclose(lm_new, G[f"lmnew_{i}"], rtol=0, atol=1e-9)
    c = face3d.split_coeff(G["semantic"][:, :257])
    assert [v.shape[1] for v in c.values()] == [80, 64, 80, 3, 27, 3]
    np.testing.assert_array_equal(np.concatenate(list(c.values()), 1), G["semantic"][:, :257])
    assert np.allclose(face3d.lm3d_from_68(np.arange(204.0).reshape(68, 3))[2], [90, 91, 92])   # nose = point 31


def test_recon_state_dict_layout_and_loader(tmp_path):
    from s2v_amd import models
    with open(os.path.join(HERE, "golden", "recon_keys.json")) as f:
        ref = json.load(f)
    net = models.define_net_recon("resnet50", use_last_fc=False, init_path="")
    assert {k: list(v.shape) for k, v in net.state_dict().items()} == ref
    sd = synth_sd("recon")
    torch.save({"net_recon": sd}, tmp_path / "face3d.pth")
    m = models.load_face3d_net(str(tmp_path / "face3d.pth"), "cpu")
    assert not m.training and torch.equal(m.state_dict()["final_layers.6.bias"], sd["final_layers.6.bias"])
    with pytest.raises(RuntimeError, match="HIP device only"):
        m(torch.zeros(1, 3, 224, 224))
    with pytest.raises(NotImplementedError):
        models.define_net_recon("resnet18")
