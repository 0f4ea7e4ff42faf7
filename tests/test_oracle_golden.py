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
