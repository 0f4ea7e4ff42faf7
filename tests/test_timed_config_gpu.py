"""The benchmarked configurations against the CPU oracle.

bench.py's headline step is ENet(+LNet) on B=16 256x256 crops as one captured HIP graph replayed back to
back, with everything the default build turns on: the FFC and encoder side streams, the style encoder
on half the CUs (grid cap, conv_igemm_x3_persist), the polyphase x2 StyleConv, the fused ToRGB and the
f16x3 arithmetic with its calibrated range guard.  These tests capture the step exactly as bench.py does
(runtime.GraphRunner over the module call), replay it several times and compare frames of the replayed
output with oracle/nets.py at SURVEY.md §8d's bar and the f16x3 bounds of tests/test_models_gpu.py; and
the same for one full-batch graph-replayed LipSyncPipeline batch against oracle/pipeline.py
(inference.py:259-288)."""
import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import synth_sd
from s2v_amd import ops, synth
from test_models_gpu import BAR, TOL, clamp01, within

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _enet():
    from s2v_amd import models
    m = models.ENet()
    m.load_state_dict(synth_sd("enet"), strict=True)
    return m.eval()


def test_lipsync_b16_graph_replay_vs_oracle():
    """B=16 ENet(+LNet) captured as bench.py captures it, replayed 3 times: 4 frames (first and last
    two) of the last replay against the oracle, every replay identical (no noise at the synthetic
    weights), and the capture took the benchmarked kernels (persistent style-encoder launches)."""
    from oracle import nets
    from s2v_amd.runtime import GraphRunner
    if ops.PRECISION != "f16x3":
        pytest.skip("the benchmarked arithmetic is f16x3")
    model = _enet()
    mel, face, gt = synth.lipsync_inputs("enet.b16", 16, 256)
    inputs = [torch.from_numpy(a).to(DEV) for a in (mel, face, gt)]
    syms = []

    def hook(ctx, p, flops, launch):
        syms.append(ops.plan_symbol(p.plan))
        launch()
    ops.CONV_HOOK = hook
    try:
        runner = GraphRunner(lambda m, f, g: model(m, f, g), inputs, warmup=1)
    finally:
        ops.CONV_HOOK = None
    assert any(s.startswith("void s2v::conv_igemm_x3_persist<256, 256,") for s in syms), "style encoder grid cap"
    outs, lows = [], []
    for _ in range(3):
        out, low = runner.replay()
        outs.append(out.clone())
        lows.append(low.clone())
    torch.cuda.synchronize()
    for o, lo in zip(outs[1:], lows[1:]):
        assert torch.equal(o, outs[0]) and torch.equal(lo, lows[0])
    idx = [0, 1, 14, 15]
    sd = synth_sd("enet")
    with torch.no_grad():
        ro, rl = nets.enet_forward(sd, torch.from_numpy(mel[idx]), torch.from_numpy(face[idx]),
                                   torch.from_numpy(gt[idx]))
    got = outs[-1][idx]
    within(clamp01(got), clamp01(ro), BAR, "replayed b16 clamped bar")
    within(got, ro, TOL["f16x3"]["enet"], "replayed b16 out")
    # LNet's B=16 output inside the replayed step (ENet.forward's ``low``: the 96x96 LNet frames)
    within(lows[-1][idx], rl, TOL["f16x3"]["low"], "replayed b16 low")


def test_lipsync_b16_noise_on_graph_replay_vs_oracle():
    """The timed configuration with StyleConv noise ON (bench.py's lipsync weights: every
    StyleConv's NoiseInjection weight 0.1, as real checkpoints carry non-zero strengths and
    base_blocks.py:528-531 draws fresh noise per call): B=16 captured as bench.py captures it,
    replayed 3 times.  Each replay draws fresh noise (outputs differ); the noise planes the last
    replay drew are read back and fed to the oracle as explicit noise tensors, and frames 0, 1,
    14, 15 of that replay must match it at the bounds of the noise-free test."""
    from oracle import nets
    from s2v_amd import models
    from s2v_amd.models import arch
    from s2v_amd.runtime import GraphRunner
    if ops.PRECISION != "f16x3":
        pytest.skip("the benchmarked arithmetic is f16x3")
    sd = synth.synth_torch_state_dict(arch.ENetParams(lnet=arch.LNetParams()), noise_weight=0.1)
    model = models.ENet()
    model.load_state_dict(sd, strict=True)
    model.eval()
    mel, face, gt = synth.lipsync_inputs("enet.b16", 16, 256)
    inputs = [torch.from_numpy(a).to(DEV) for a in (mel, face, gt)]
    runner = GraphRunner(lambda m, f, g: model(m, f, g), inputs, warmup=1)
    eng = model._engine(inputs[0].device)[0]
    outs = []
    for _ in range(3):
        outs.append(runner.replay()[0].clone())
    torch.cuda.synchronize()
    assert (outs[1] - outs[2]).abs().max() > 1e-3, "every replay draws fresh noise"
    assert all(n is not None for n in eng.last_noises)
    idx = [0, 1, 14, 15]
    noises = [n[idx].cpu().unsqueeze(1) for n in eng.last_noises]
    assert [tuple(n.shape[2:]) for n in noises] == [(200, 200), (200, 200), (400, 400), (400, 400)]
    for n in noises:                                   # N(0, 1) draws
        assert abs(float(n.mean())) < 0.02 and 0.95 < float(n.std()) < 1.05
    with torch.no_grad():
        ro, _ = nets.enet_forward(sd, torch.from_numpy(mel[idx]), torch.from_numpy(face[idx]),
                                  torch.from_numpy(gt[idx]), noises=noises)
    got = outs[-1][idx]
    within(clamp01(got), clamp01(ro), BAR, "replayed b16 noise-on clamped bar")
    within(got, ro, TOL["f16x3"]["enet"], "replayed b16 noise-on out")


def test_lnet_bench_capture_vs_oracle():
    """configs[1] as bench.py times it (bench.LNetOnly: the device bilinear resize of B=16 256x256
    crops to 96x96, then LNet.forward, captured by runtime.GraphRunner with warmup 1 and replayed):
    frames 0, 1, 14, 15 of the third replay against oracle.nets.lnet_forward on F.interpolate'd crops,
    at the LNet bounds of tests/test_models_gpu.py.  The pre-sigmoid logits are captured in the same
    graph (the engine's ``logits=`` output: one more 7x7 conv at the end) and compared too."""
    import argparse

    import torch.nn.functional as F

    import bench
    from oracle import nets
    from s2v_amd.ops import NHWC
    from s2v_amd.runtime import GraphRunner
    if ops.PRECISION != "f16x3":
        pytest.skip("the benchmarked arithmetic is f16x3")
    args = argparse.Namespace(batch=16, size=256, lanes=1)
    wl = bench.LNetOnly(args, torch.device(DEV, torch.cuda.current_device()), 0)
    eng = wl.model._engine(wl.inputs[1].device)[0]
    logits = NHWC.empty(16, 96, 96, 3, DEV)
    orig = eng.forward
    eng.forward = lambda ctx, a, f, o, logits_=None, pad_rgb=False: orig(ctx, a, f, o, logits=logits, pad_rgb=pad_rgb)
    try:
        runner = GraphRunner(lambda *x: wl.fn_lane(0, *x), list(wl.inputs), warmup=1)
    finally:
        del eng.forward
    outs, lgs = [], []
    for _ in range(3):
        outs.append(runner.replay().clone())
        lgs.append(logits.t.clone())
    torch.cuda.synchronize()
    for o, lg in zip(outs[1:], lgs[1:]):
        assert torch.equal(o, outs[0]) and torch.equal(lg, lgs[0])
    idx = [0, 1, 14, 15]
    mel = wl.inputs[0][idx].cpu()
    f96 = F.interpolate(wl.inputs[1][idx].cpu(), (96, 96), mode="bilinear", align_corners=False)
    with torch.no_grad():
        ro, aux = nets.lnet_forward(wl.sd, mel, f96, return_aux=True)
    within(outs[-1][idx], ro, BAR, "lnet bench clamped bar")
    within(outs[-1][idx], ro, TOL["f16x3"]["lnet"], "lnet bench out")
    within(lgs[-1][idx].permute(0, 3, 1, 2), aux["logits"], TOL["f16x3"]["logits"], "lnet bench logits")


def test_pipeline_full_batch_graph_replay_vs_oracle():
    """One full 16-frame LipSyncPipeline batch (DNet -> uint8 ref -> ENet(+LNet) -> uint8) as a
    replayed graph, run twice: frames 0, 1 and 15 against oracle/pipeline.py at the uint8 bar of
    tests/test_pipeline_gpu.py, and the second run equal to the first."""
    from oracle import pipeline as OP
    from s2v_amd import audio, models, pipeline as P
    from test_pipeline_gpu import _check_u8, _clip
    d = models.DNet()
    d.load_state_dict(synth_sd("dnet"), strict=True)
    dnet, enet = d.eval(), _enet()
    wav, semantic, expression, src = _clip(16, 9)
    chunks = audio.mel_chunks(audio.melspectrogram(torch.from_numpy(wav).to(DEV)))
    n = min(chunks.shape[0], 16)
    assert n == 16
    coeffs = torch.from_numpy(P.dnet_coefficients(semantic[:n], expression))
    pipe = P.LipSyncPipeline(dnet, enet, DEV, batch=16)
    got = pipe.run(chunks, src[:n].to(DEV), coeffs.to(DEV), 0, n)
    again = pipe.run(chunks, src[:n].to(DEV), coeffs.to(DEV), 0, n)
    assert pipe._runner is not None and pipe.reruns == 0
    assert torch.equal(got.cpu(), again.cpu())
    idx = [0, 1, 15]
    with torch.no_grad():
        ref = OP.lipsync_frames(synth_sd("dnet"), synth_sd("enet"), chunks[idx].cpu(), src[idx], coeffs[idx])
    _check_u8(got[idx], ref)
    assert np.isfinite(got.float().cpu().numpy()).all()
