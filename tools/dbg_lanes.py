#!/usr/bin/env python3
"""Debug: graph replays of ENet — sequential repeats and two graphs replayed concurrently on two
streams.  Prints how many of DBG_REPS concurrent rounds differ from the sequential replays.
Env: DBG_B (batch), DBG_REPS, DBG_EAGER=1 (an eager forward of m1 between the phases)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from helpers import synth_sd  # noqa: E402
from s2v_amd import models, synth  # noqa: E402
from s2v_amd.runtime import GraphRunner  # noqa: E402

B = int(os.environ.get("DBG_B", "4"))
REPS = int(os.environ.get("DBG_REPS", "12"))
dev = "cuda"
tag = " ".join(f"{k}={os.environ[k]}" for k in ("S2V_ENET_OVERLAP", "S2V_LNET_BRANCHES") if k in os.environ) or "default"


def enet():
    sd = {k: (torch.zeros_like(v) if k.startswith("style_convs.") and k.endswith(".weight") and v.numel() == 1
              else v) for k, v in synth_sd("enet").items()}
    m = models.ENet()
    m.load_state_dict(sd)
    return m.eval()


def inputs(t):
    return [torch.from_numpy(a).to(dev) for a in synth.lipsync_inputs(t, B, 256)]


def diff(a, b):
    return max(float((x - y).abs().max()) for x, y in zip(a, b))


m1, m2 = enet(), enet()
r1 = GraphRunner(lambda *a: m1(*a), inputs("a"), warmup=1)
r2 = GraphRunner(lambda *a: m2(*a), inputs("b"), warmup=1)
torch.cuda.synchronize()
base = []
for r in (r1, r2):
    r.replay()
    torch.cuda.synchronize()
    base.append([t.clone() for t in r.static_out])
seq_bad = 0
for k in range(4):
    r1.replay()
    torch.cuda.synchronize()
    seq_bad += diff(r1.static_out, base[0]) != 0
if os.environ.get("DBG_EAGER") == "1":
    eager = m1(*r1.static_in)
    torch.cuda.synchronize()
    print(f"[{tag}] eager forward vs r1 replay: {diff(eager, base[0]):.3e}", flush=True)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
cur = torch.cuda.current_stream()
bad = []
for rep in range(REPS):
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        r1.replay()
    with torch.cuda.stream(s2):
        r2.replay()
    cur.wait_stream(s1)
    cur.wait_stream(s2)
    torch.cuda.synchronize()
    d1, d2 = diff(r1.static_out, base[0]), diff(r2.static_out, base[1])
    if d1 or d2:
        bad.append((rep, f"{d1:.2e}", f"{d2:.2e}"))
# same two graphs, alternating on one stream
alt_bad = 0
for rep in range(4):
    r1.replay()
    r2.replay()
    torch.cuda.synchronize()
    alt_bad += (diff(r1.static_out, base[0]) != 0) + (diff(r2.static_out, base[1]) != 0)
print(f"[{tag}] sequential bad {seq_bad}/4, concurrent bad {len(bad)}/{REPS} {bad[:6]}, alternating bad {alt_bad}/8",
      flush=True)
