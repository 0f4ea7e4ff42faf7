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
    outs = []
    for _ in range(3):
        out, _low = runner.replay()
        outs.append(out.clone())
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    idx = [0, 1, 14, 15]
    sd = synth_sd("enet")
    with torch.no_grad():
        ro, _ = nets.enet_forward(sd, torch.from_numpy(mel[idx]), torch.from_numpy(face[idx]),
                                  torch.from_numpy(gt[idx]))
    got = outs[-1][idx]
    within(clamp01(got), clamp01(ro), BAR, "replayed b16 clamped bar")
    within(got, ro, TOL["f16x3"]["enet"], "replayed b16 out")


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
