"""Noise injection on the device (SURVEY.md §8a StyleConv / GFPGAN rows, Appendix B "random noise").

* Parity with explicit noise tensors and NON-ZERO noise strengths (real checkpoints have w != 0;
  the synthetic fixtures keep the init value 0): ENet StyleConv out + w * noise
  (base_blocks.py:524-536) and GFPGAN StyleConv (stylegan2_clean_arch.py:126-134) against the CPU
  oracle with the same noise tensors.
* randomize semantics: the reference draws normal_() per call; the engines draw from a
  counter-based generator whose offset advances through a device-side counter bumped inside the
  forward, so an eager call AND every replay of a captured HIP graph draw fresh noise.
"""
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import GFPGAN_KW, max_abs, synth_sd
from s2v_amd import synth

pytestmark = pytest.mark.gpu
DEV = "cuda"
NOISE_W = (0.1, -0.2, 0.15, 0.05)


def _enet_sd():
    sd = dict(synth_sd("enet"))
    for i, w in enumerate(NOISE_W):
        sd[f"style_convs.{i}.weight"] = torch.tensor([w])
    return sd


def _enet(sd):
    from s2v_amd import models
    m = models.ENet()
    m.load_state_dict(sd, strict=True)
    return m.eval()


def _enet_noises(b, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(b, 1, s, s, generator=g) for s in (200, 200, 400, 400)]


def test_enet_explicit_noise_matches_oracle(prec):
    from oracle import nets
    from test_models_gpu import TOL
    sd = _enet_sd()
    enet = _enet(sd)
    mel, face, gt = synth.lipsync_inputs("noise.enet", 2, 256)
    noises = _enet_noises(2, 5)
    out, _ = enet(*(torch.from_numpy(a).to(DEV) for a in (mel, face, gt)),
                  noises=[n.to(DEV).reshape(2, n.shape[2], n.shape[3]) for n in noises])
    with torch.no_grad():
        ref, _ = nets.enet_forward(sd, *(torch.from_numpy(a) for a in (mel, face, gt)), noises=noises)
    m, mean = max_abs(out, ref)
    assert m <= TOL[prec]["enet"][0] and mean <= TOL[prec]["enet"][1], (m, mean)
    # the noise term is really there: the zero-noise forward differs by ~|w| * |noise|
    out0, _ = enet(*(torch.from_numpy(a).to(DEV) for a in (mel, face, gt)),
                   noises=[torch.zeros(2, n.shape[2], n.shape[3], device=DEV) for n in noises])
    assert (out - out0).abs().max() > 1e-2


def test_enet_random_noise_fresh_per_call_and_replay():
    from s2v_amd.runtime import GraphRunner
    enet = _enet(_enet_sd())
    mel, face, gt = (torch.from_numpy(a).to(DEV) for a in synth.lipsync_inputs("noise.enet.r", 2, 256))
    a, _ = enet(mel, face, gt)
    b, _ = enet(mel, face, gt)
    assert torch.isfinite(a).all() and (a - b).abs().max() > 1e-3
    runner = GraphRunner(lambda m, f, g: enet(m, f, g)[0], [mel, face, gt], warmup=1)
    r1 = runner.replay().clone()
    r2 = runner.replay().clone()
    assert (r1 - r2).abs().max() > 1e-3, "graph replays must draw fresh noise"
    # and the draws are N(0,1)-scaled: the replay spread matches the eager one
    s_eager, s_graph = float((a - b).std()), float((r1 - r2).std())
    assert 0.5 < s_graph / s_eager < 2.0, (s_eager, s_graph)


def test_gfpgan_explicit_noise_matches_oracle():
    from oracle import enhancers
    from s2v_amd import models
    sd = synth_sd("gfpgan")
    m = models.GFPGANv1Clean(**GFPGAN_KW)
    m.load_state_dict(sd, strict=True)
    eng, ctx = m._engine(torch.device(DEV))
    x = torch.from_numpy(synth.face_inputs("noise.gfpgan", 1))
    g = torch.Generator().manual_seed(9)
    noises = [torch.randn(1, 1, 2 ** ((j + 5) // 2), 2 ** ((j + 5) // 2), generator=g) for j in range(2 * eng.levels + 1)]
    out = torch.empty((1, 3, 512, 512), device=DEV)
    eng.forward(ctx, x.to(DEV), out, return_rgb=False, noises=[n.to(DEV) for n in noises])
    with torch.no_grad():
        ref, _, _ = enhancers.gfpgan_forward(sd, x, noises=noises, return_rgb=False)
    m_, mean = max_abs(out, ref)
    scale = float(ref.abs().max())
    assert m_ < 1e-3 * scale and mean < 1e-4 * scale, (m_, mean, scale)


def test_gfpgan_random_noise_fresh_per_replay():
    from s2v_amd import models
    from s2v_amd.runtime import GraphRunner
    m = models.GFPGANv1Clean(**GFPGAN_KW)
    m.load_state_dict(synth_sd("gfpgan"), strict=True)
    x = torch.from_numpy(synth.face_inputs("noise.gfpgan.r", 1)).to(DEV)
    runner = GraphRunner(lambda t: m(t, return_rgb=False)[0], [x], warmup=1)
    r1 = runner.replay().clone()
    r2 = runner.replay().clone()
    assert torch.isfinite(r1).all() and (r1 - r2).abs().max() > 0
