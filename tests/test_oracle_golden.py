"""The CPU oracle restatement (oracle/nets.py) against goldens produced by the reference itself.

Tolerances: the fp32-vs-fp64 spread of the reference on these nets is 5e-4..7e-4,
and the oracle is the same math at fp32 with different op grouping, so per-tensor bounds are set
at about that spread scaled by each tensor's magnitude.
"""
import numpy as np
import torch

from oracle import nets
from helpers import synth_sd, max_abs, check_probe
from s2v_amd import synth


def test_lnet_oracle_matches_reference(golden):
    g = golden("lnet_b2_96")
    sd = synth_sd("lnet")
    mel, face, _ = synth.lipsync_inputs("golden.lnet", 2, 96)
    with torch.no_grad():
        out, aux = nets.lnet_forward(sd, torch.from_numpy(mel), torch.from_numpy(face), return_aux=True)
    assert max_abs(aux["audio_feat"], g["audio_feat"])[0] < 1e-3
    for i, t in enumerate(aux["enc"]):
        check_probe(t, g, f"enc{i}", atol=1e-4, rtol=1e-4)
    m, mean = max_abs(aux["logits"], g["logits"])
    assert m < 2e-3 and mean < 1e-4, (m, mean)
    m, mean = max_abs(out, g["out"])
    assert m < 5e-4 and mean < 3e-5, (m, mean)


def test_enet_oracle_matches_reference(golden):
    sd = synth_sd("enet")
    for size in (256, 384):
        g = golden(f"enet_b1_{size}")
        mel, face, gt = synth.lipsync_inputs(f"golden.enet{size}", 1, size)
        with torch.no_grad():
            out, low, aux = nets.enet_forward(sd, torch.from_numpy(mel), torch.from_numpy(face),
                                              torch.from_numpy(gt), return_aux=True)
        assert max_abs(aux["style"], g["style"])[0] < 1e-3
        assert max_abs(low, g["low"])[0] < 5e-4
        if "out" in g.files:
            m, mean = max_abs(out, g["out"])
            assert m < 5e-3 and mean < 2e-4, (m, mean)
        else:
            check_probe(out, g, "out", atol=5e-3)


def test_dnet_oracle_matches_reference(golden):
    sd = synth_sd("dnet")
    for size, batch in ((128, 2), (256, 1)):
        g = golden(f"dnet_b{batch}_{size}")
        src, coeff = synth.dnet_inputs(f"golden.dnet{size}", batch, size)
        with torch.no_grad():
            out = nets.dnet_forward(sd, torch.from_numpy(src), torch.from_numpy(coeff), return_aux=True)
        assert max_abs(out["descriptor"], g["descriptor"])[0] < 1e-4
        assert max_abs(out["flow_field"], g["flow"])[0] < 2e-4
        for k in ("warp_image", "fake_image"):
            if k in g.files:
                m, _ = max_abs(out[k], g[k])
                assert m < 2e-4, (k, m)
            else:
                check_probe(out[k], g, k, atol=2e-4)


def test_flow_warp_oracle_matches_reference(golden):
    g = golden("ops")
    flow = torch.from_numpy(synth.hash_array("golden.flow", (2, 2, 16, 16), -3.0, 3.0))
    src = torch.from_numpy(synth.hash_array("golden.flow.src", (2, 3, 64, 64)))
    assert max_abs(nets.warp_image(src, nets.flow_to_deformation(flow)), g["warp"])[0] < 1e-5
    flow2 = torch.from_numpy(synth.hash_array("golden.flow2", (1, 2, 32, 32), -2.0, 2.0))
    src2 = torch.from_numpy(synth.hash_array("golden.flow2.src", (1, 3, 32, 32)))
    assert max_abs(nets.warp_image(src2, nets.flow_to_deformation(flow2)), g["warp_same"])[0] < 1e-5


def test_gfpgan_oracle_matches_reference(golden):
    from oracle import enhancers
    g = golden("gfpgan_b1_512")
    x = torch.from_numpy(synth.face_inputs("golden.gfpgan", 1))
    with torch.no_grad():
        img, rgbs, style = enhancers.gfpgan_forward(synth_sd("gfpgan"), x)
    assert max_abs(style.reshape(1, -1), g["style"])[0] < 1e-4
    assert max_abs(rgbs[0], g["rgb0"])[0] < 1e-3 and max_abs(rgbs[3], g["rgb3"])[0] < 1e-3
    check_probe(rgbs[6], g, "rgb6", atol=1e-4, rtol=1e-4)
    check_probe(img, g, "out", atol=1e-3, rtol=1e-4)


def test_gpen_oracle_matches_reference(golden):
    from oracle import enhancers
    g = golden("gpen_b1_512")
    x = torch.from_numpy(synth.face_inputs("golden.gpen", 1))
    with torch.no_grad():
        img, lat, code = enhancers.gpen_forward(synth_sd("gpen"), x)
    assert max_abs(code, g["code"])[0] < 1e-5 and max_abs(lat, g["latent"])[0] < 1e-4
    check_probe(img, g, "out", atol=1e-4, rtol=1e-4)


def test_gpen2048_oracle_matches_reference(golden):
    """GPEN-BFR-2048 (FullGenerator(2048, 512, 8, 2), face_gan.py:26-28) restatement vs the reference."""
    import json
    import os
    from oracle import enhancers
    from s2v_amd.models.enhancer_arch import FullGeneratorParams
    with open(os.path.join(os.path.dirname(__file__), "golden", "gpen2048_keys.json")) as f:
        assert {k: list(v.shape) for k, v in FullGeneratorParams(2048, 512, 8, 2).state_dict().items()} == json.load(f)
    g = golden("gpen_b1_2048")
    x = torch.from_numpy(synth.face_inputs("golden.gpen2048", 1, 2048))
    with torch.no_grad():
        img, _, code = enhancers.gpen_forward(synth_sd("gpen2048"), x)
    assert max_abs(code, g["code"])[0] < 1e-5
    check_probe(img, g, "out", atol=1e-4, rtol=1e-4)


def test_upfirdn2d_and_fused_act_oracle_match_reference_fallbacks(golden):
    from oracle import enhancers
    g = golden("ops")
    x = torch.from_numpy(synth.hash_array("golden.fba.x", (2, 8, 5, 7)))
    b = torch.from_numpy(synth.hash_array("golden.fba.b", (8,)))
    assert max_abs(enhancers.fused_leaky_relu(x, b), g["fba_out"])[0] == 0.0
    k = torch.tensor([1.0, 3.0, 3.0, 1.0])
    k = k[None, :] * k[:, None] / 64.0
    xi = torch.from_numpy(synth.hash_array("golden.ufd.x", (2, 3, 9, 11)))
    for name, (up, down, pad) in {"up2": (2, 1, (2, 1)), "blur22": (1, 1, (2, 2)),
                                  "blur11": (1, 1, (1, 1)), "down2": (1, 2, (1, 1))}.items():
        got = enhancers.upfirdn2d(xi, k * (4 if up == 2 else 1), up=up, down=down, pad=pad)
        assert max_abs(got, g[f"ufd_{name}"])[0] < 1e-6, name


def test_parsenet_oracle_matches_reference(golden):
    from oracle import parse
    from helpers import parsenet_sd
    for size, batch in ((128, 2), (512, 1)):
        g = golden(f"parsenet_b{batch}_{size}")
        x = torch.from_numpy(synth.face_inputs(f"golden.parsenet{size}", batch, size))
        with torch.no_grad():
            mask, img = parse.parsenet_forward(parsenet_sd(size), x)
        if size == 128:
            scale = float(np.abs(g["mask"]).max())
            assert max_abs(mask, g["mask"])[0] < 1e-4 * scale and max_abs(img, g["img"])[0] < 1e-4 * scale
        else:
            check_probe(mask, g, "mask", atol=1e-4 * float(g["mask_stats"][2]))
            check_probe(img, g, "img", atol=1e-4 * float(g["img_stats"][2]))
        agree = (mask.argmax(1).numpy() == g["argmax"]).mean()
        assert agree > 0.9999, agree


def test_rrdbnet_oracle_matches_reference(golden):
    """oracle/sr.py vs the reference RRDBNet forward (rrdbnet_arch.py) and RealESRNet.process
    (real_esrnet.py:99-137, incl. reflect padding, tiling and the uint8 rounding) run unmodified."""
    from helpers import RRDB_FORWARD, RRDB_PROCESS, rrdb_sd
    from oracle import sr
    g = golden("rrdbnet_goldens")
    for tag, scale, shape in RRDB_FORWARD:
        x = torch.from_numpy(synth.hash_array(f"golden.rrdb.{tag}", shape, 0.0, 1.0))
        with torch.no_grad():
            y = sr.rrdbnet_forward(rrdb_sd(scale), x, scale).numpy()
        ref = g[f"fwd_{tag}"]
        assert y.shape == ref.shape
        assert np.abs(y - ref).max() <= 1e-4 * np.abs(ref).max(), tag
    for tag, scale, h, w, tile, pad in RRDB_PROCESS:
        img = synth.sr_frame(f"golden.rrdb.{tag}", 1, h, w)[0]
        out = sr.realesrnet_process(rrdb_sd(scale), img, scale, tile, pad)
        ref = g[f"proc_{tag}"]
        # the reference crops only h_pad / w_pad rows / columns off the *upscaled* output
        # (real_esrnet.py:126-128), so an odd 27x31 frame at x2 gives 55x63, not 54x62
        hp, wp = (-h) % {2: 2, 1: 4}.get(scale, 1), (-w) % {2: 2, 1: 4}.get(scale, 1)
        assert out.shape == ref.shape == ((h + hp) * scale - hp, (w + wp) * scale - wp, 3)
        assert (np.abs(out.astype(int) - ref.astype(int)) <= 1).all() and (out != ref).mean() <= 1e-3, tag


def test_rrdbnet_state_dict_layout_matches_reference():
    """models.sr_arch.RRDBNetParams has the reference's RRDBNet keys and shapes (manifests written by
    make_golden.py from the reference modules) for every scale."""
    import json
    import os
    from s2v_amd.models.sr_arch import RRDBNetParams
    here = os.path.join(os.path.dirname(__file__), "golden")
    for scale, name in ((2, "rrdbnet"), (4, "rrdbnet_x4"), (1, "rrdbnet_x1")):
        with open(os.path.join(here, f"{name}_keys.json")) as f:
            ref = json.load(f)
        mine = {k: list(v.shape) for k, v in RRDBNetParams(3, 3, scale=scale, num_feat=32).state_dict().items()}
        assert mine == ref
