#!/usr/bin/env python3
"""Debug: tests/test_lanes_gpu.py::test_lanes_of_one_module_and_a_shallow_copy with diagnostics.
Which runner's frames differ after concurrent replays, by how much, and where.
Env: DBG_CASE = lanes | peer | both (default both), DBG_REPS (concurrent rounds)."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from helpers import synth_sd  # noqa: E402
from s2v_amd import models, synth  # noqa: E402
from s2v_amd.runtime import GraphRunner, LaneRunner  # noqa: E402

B = 4
dev = "cuda"
CASE = os.environ.get("DBG_CASE", "both")
REPS = int(os.environ.get("DBG_REPS", "4"))
tag = " ".join(f"{k}={os.environ[k]}" for k in ("S2V_ENET_OVERLAP", "S2V_LNET_BRANCHES", "DBG_CASE")
               if k in os.environ) or "default"


def enet():
    sd = {k: (torch.zeros_like(v) if k.startswith("style_convs.") and k.endswith(".weight") and v.numel() == 1
              else v) for k, v in synth_sd("enet").items()}
    m = models.ENet()
    m.load_state_dict(sd)
    return m.eval()


def inputs(seed):
    return [torch.from_numpy(a).to(dev) for a in synth.lipsync_inputs(f"lanes{seed}", B, 256)]


def report(name, got, ref):
    out = []
    for i, (g, r) in enumerate(zip(got, ref)):
        d = (g - r).abs()
        nz = int((d != 0).sum())
        if nz:
            idx = (d != 0).nonzero()
            out.append(f"out{i}: {nz}/{d.numel()} differ, max {float(d.max()):.3e}, samples "
                       f"{sorted(set(idx[:, 0].tolist()))}, rows {int(idx[:, 2].min())}..{int(idx[:, 2].max())}")
    print(f"  [{tag}] {name}: {'OK' if not out else '; '.join(out)}", flush=True)
    return not out


m = enet()
runners, names = [], []
if CASE in ("lanes", "both"):
    x1, x2 = inputs(3), inputs(4)
    lanes = LaneRunner(lambda lane, *a: m(*a, lane=lane), x1, lanes=2, warmup=1)
    for i in range(3):
        lanes.runners[1].static_in[i].copy_(x2[i])
    runners += lanes.runners
    names += ["lane0", "lane1"]
if CASE in ("peer", "both"):
    peer = copy.copy(m)
    rp = GraphRunner(lambda *a: peer(*a), inputs(5), warmup=1)
    runners.append(rp)
    names.append("peer")
    if CASE == "peer":
        r0 = GraphRunner(lambda *a: m(*a), inputs(3), warmup=1)
        runners.insert(0, r0)
        names.insert(0, "m")
seq = []
for r in runners:
    r.replay()
    torch.cuda.synchronize()
    seq.append(tuple(t.clone() for t in r.static_out))
# sequential repeat
for r, s, n in zip(runners, seq, names):
    r.replay()
    torch.cuda.synchronize()
    report(n + " seq-repeat", r.static_out, s)
streams = [torch.cuda.Stream() for _ in runners]
cur = torch.cuda.current_stream()
for rep in range(REPS):
    for st in streams:
        st.wait_stream(cur)
    for r, st in zip(runners, streams):
        with torch.cuda.stream(st):
            r.replay()
    for st in streams:
        cur.wait_stream(st)
    torch.cuda.synchronize()
    for r, s, n in zip(runners, seq, names):
        report(f"{n} concurrent#{rep}", r.static_out, s)
# after: sequential again (is the damage persistent state?)
for r, s, n in zip(runners, seq, names):
    r.replay()
    torch.cuda.synchronize()
    report(n + " seq-after", r.static_out, s)
