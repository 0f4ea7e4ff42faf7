#!/usr/bin/env python3
"""Debug: first layer whose output differs between sequential and concurrent replays of two lanes
of one ENet module (tools/dbg_lanes3.py: f16x3 only, no side streams needed).  Every conv /
norm / resize output is copied into a probe buffer inside the captured graph."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from helpers import synth_sd  # noqa: E402
from s2v_amd import models, ops, synth  # noqa: E402
from s2v_amd.runtime import GraphRunner  # noqa: E402

dev = "cuda"
B = 4
REPS = int(os.environ.get("DBG_REPS", "4"))
PROBES = {}          # lane -> list of (name, probe tensor)
CUR = [None]

orig_run_conv = ops._run_conv


def run_conv(ctx, launch, x, cw, yv, pool, *a, **k):
    orig_run_conv(ctx, launch, x, cw, yv, pool, *a, **k)
    if CUR[0] is not None:
        CUR[0].append((f"conv {tuple(x.v.shape)}->{tuple(yv.shape)} k{cw.kh} s{cw.sh} pool{int(pool)}", yv.clone()))


ops._run_conv = run_conv


def wrap(name, argi):
    f = getattr(ops, name)

    def g(*a, **k):
        r = f(*a, **k)
        if CUR[0] is not None:
            t = a[argi]
            t = t.v if isinstance(t, ops.NHWC) else t
            CUR[0].append((f"{name} {tuple(t.shape)}", t.clone()))
        return r
    setattr(ops, name, g)


for n, i in (("resize_nhwc", 2), ("layernorm2d", 4), ("instnorm", 2), ("pad_reflect", 2), ("modconv_demod", 3),
             ("nchw_to_nhwc", 2), ("rfft2", 3), ("irfft2", 3), ("attention", 4), ("row_layernorm", 4)):
    wrap(n, i)

sd = {k: (torch.zeros_like(v) if k.startswith("style_convs.") and k.endswith(".weight") and v.numel() == 1
          else v) for k, v in synth_sd("enet").items()}
m = models.ENet()
m.load_state_dict(sd)
m.eval()


class Probed(GraphRunner):
    def __init__(self, lane, x):
        self.lane = lane
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            m(*x, lane=lane)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.static_in = [t.clone() for t in x]
        self.graph = torch.cuda.CUDAGraph()
        PROBES[lane] = []
        CUR[0] = PROBES[lane]
        with torch.cuda.graph(self.graph):
            self.static_out = m(*self.static_in, lane=lane)
        CUR[0] = None
        torch.cuda.synchronize()


rs = [Probed(lane, [torch.from_numpy(a).to(dev) for a in synth.lipsync_inputs(f"lanes{lane}", B, 256)])
      for lane in range(2)]
print(f"{len(PROBES[0])} probes per lane", flush=True)


def snap(lane):
    return [t.clone() for _, t in PROBES[lane]]


seq = []
for r in rs:
    r.replay()
    torch.cuda.synchronize()
    seq.append(snap(r.lane))
streams = [torch.cuda.Stream() for _ in rs]
cur = torch.cuda.current_stream()
for rep in range(REPS):
    for st in streams:
        st.wait_stream(cur)
    for r, st in zip(rs, streams):
        with torch.cuda.stream(st):
            r.replay()
    for st in streams:
        cur.wait_stream(st)
    torch.cuda.synchronize()
    for r in rs:
        now = snap(r.lane)
        first = None
        for i, (a, b) in enumerate(zip(now, seq[r.lane])):
            if not torch.equal(a, b):
                d = (a - b).abs()
                nz = (d != 0).nonzero()
                ix = [tuple(v) for v in nz[:4].tolist()]
                vals = [(float(a[v]), float(b[v]), hex(int(a[v].view(torch.int32)) & 0xffffffff)) for v in ix]
                first = (f"probe {i} '{PROBES[r.lane][i][0]}': {int((d != 0).sum())}/{d.numel()} differ, max "
                         f"{float(d.nan_to_num(1e30).max()):.3e}, nan {int(torch.isnan(a).sum())}, first idx "
                         f"{ix} (now, seq, now-bits) {vals}")
                break
        print(f"  rep {rep} lane {r.lane}: {first or 'OK'}", flush=True)
