"""Concurrent execution of captured forwards.

Round 2 saw two 16-frame batches replayed concurrently on two streams corrupt each other's frames.
The cause: every piece of mutable device state of a forward — the split-K / norm workspaces, the
LNet FFC branch streams and their workspaces, ENet's style-encoder side stream, the noise draw
counter and the ADAIN parameter tensor (kept on the shared AdainBank) — hung off the engine or the
module (``_s2v_engines``), and a peer copy of a module (copy.copy) shares that dict.  Two graphs
captured through the same engine bake the same workspace addresses; replayed at the same time they
write them concurrently.  That state now lives in a per-lane ``ops.Ctx`` (engines keep only
read-only weights), and module copies get fresh engines (``_EngineMixin.__getstate__``).

These tests replay graphs concurrently on two streams and require every output bit to equal the
sequential replays: two independently built ENet modules, two lanes of one module, a shallow copy
of a module, and the full DNet -> ENet pipeline on lanes against its one-lane run."""
import copy

import pytest
import torch

import s2v_import  # noqa: F401
from helpers import synth_sd
from s2v_amd import models, synth
from s2v_amd.runtime import GraphRunner, LaneRunner

pytestmark = pytest.mark.gpu
DEV = "cuda"
B = 4


def _enet():
    # StyleConv noise weight 0 (the reference's init value, base_blocks.py:528): the frames are then a
    # function of the inputs alone, whatever the replay count of each lane's noise counter
    sd = {k: (torch.zeros_like(v) if k.startswith("style_convs.") and k.endswith(".weight") and v.numel() == 1
              else v) for k, v in synth_sd("enet").items()}
    m = models.ENet()
    m.load_state_dict(sd, strict=True)
    return m.eval()


def _inputs(seed):
    return [torch.from_numpy(a).to(DEV) for a in synth.lipsync_inputs(f"lanes{seed}", B, 256)]


def _concurrent(runners, streams, reps=3):
    """Replay every runner ``reps`` times, runner i on streams[i], with no ordering between them."""
    cur = torch.cuda.current_stream()
    for st in streams:
        st.wait_stream(cur)
    for _ in range(reps):
        for r, st in zip(runners, streams):
            with torch.cuda.stream(st):
                r.replay()
    for st in streams:
        cur.wait_stream(st)
    torch.cuda.synchronize()
    return [tuple(t.clone() for t in r.static_out) for r in runners]


def _same(a, b):
    return all(torch.equal(x, y) for x, y in zip(a, b))


def test_two_modules_replayed_concurrently_match_sequential():
    m1, m2 = _enet(), _enet()
    x1, x2 = _inputs(1), _inputs(2)
    r1 = GraphRunner(lambda *a: m1(*a), x1, warmup=1)
    r2 = GraphRunner(lambda *a: m2(*a), x2, warmup=1)
    seq = []
    for r in (r1, r2):
        r.replay()
        torch.cuda.synchronize()
        seq.append(tuple(t.clone() for t in r.static_out))
    assert not torch.equal(seq[0][0], seq[1][0])               # different inputs, different frames
    got = _concurrent([r1, r2], [torch.cuda.Stream(), torch.cuda.Stream()])
    assert _same(got[0], seq[0]) and _same(got[1], seq[1])


def test_lanes_of_one_module_and_a_shallow_copy():
    m = _enet()
    peer = copy.copy(m)                      # the round-2 "peer copy": must not share engines / lanes
    x1, x2, x3 = _inputs(3), _inputs(4), _inputs(5)
    lanes = LaneRunner(lambda lane, *a: m(*a, lane=lane), x1, lanes=2, warmup=1)
    lanes.runners[1].static_in[0].copy_(x2[0])
    lanes.runners[1].static_in[1].copy_(x2[1])
    lanes.runners[1].static_in[2].copy_(x2[2])
    rp = GraphRunner(lambda *a: peer(*a), x3, warmup=1)
    assert m.__dict__["_s2v_engines"] is not peer.__dict__["_s2v_engines"]
    runners = [lanes.runners[0], lanes.runners[1], rp]
    seq = []
    for r in runners:
        r.replay()
        torch.cuda.synchronize()
        seq.append(tuple(t.clone() for t in r.static_out))
    got = _concurrent(runners, [torch.cuda.Stream() for _ in runners], reps=4)
    for g, s in zip(got, seq):
        assert _same(g, s)
    # and through the round-robin LaneRunner itself
    for _ in range(5):
        lanes.replay()
    torch.cuda.synchronize()
    assert _same(lanes.runners[0].static_out, seq[0]) and _same(lanes.runners[1].static_out, seq[1])


def test_pipeline_on_two_lanes_equals_one_lane():
    from s2v_amd import pipeline as P
    d = models.DNet()
    d.load_state_dict(synth_sd("dnet"), strict=True)
    e = _enet()
    n = 3 * B + 1                                  # three graph batches over two lanes + an eager tail
    g = torch.Generator(device=DEV).manual_seed(11)
    mel = torch.rand((n, 1, 80, 16), generator=g, device=DEV) * 8 - 4
    src = torch.rand((n, 3, 256, 256), generator=g, device=DEV) * 2 - 1
    coeff = torch.randn((n, 73, 26), generator=g, device=DEV)
    one = P.LipSyncPipeline(d.eval(), e, DEV, batch=B, lanes=1).run(mel, src, coeff)
    two = P.LipSyncPipeline(copy.copy(d), copy.copy(e), DEV, batch=B, lanes=2).run(mel, src, coeff)
    torch.cuda.synchronize()
    assert torch.equal(one, two)


def _pool_of(t):
    addr = t.data_ptr()
    for seg in torch.cuda.memory_snapshot():
        if seg["address"] <= addr < seg["address"] + seg["total_size"]:
            return tuple(seg.get("segment_pool_id", (0, 0)))
    return None


def test_side_branch_allocations_are_graph_owned():
    """ops.side_stream: a side branch's tensors come from the capture stream, so they belong to the
    captured graph's private pool.  (A plain allocation on the forked side stream is reported as
    well: on ROCm it is the one the round-2 corruption came from.)"""
    from s2v_amd import ops
    side = torch.cuda.Stream()
    keep = []
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            raw = torch.empty(1 << 20, device=DEV)
            raw.fill_(1.0)
        with ops.side_stream(side, keep):
            ours = ops.empty((1 << 20,), DEV)
            ours.fill_(2.0)
        main_t = torch.empty(1 << 20, device=DEV)
        main_t.fill_(3.0)
        cur.wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    pm, po, pr = _pool_of(main_t), _pool_of(ours), _pool_of(raw)
    print(f"pools: capture stream {pm}, side_stream() {po}, plain side-stream allocation {pr}")
    assert pm is not None and pm != (0, 0) and po == pm and keep and keep[0] is ours
