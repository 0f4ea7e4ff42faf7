#!/usr/bin/env python3
"""Debug bisect of the lane corruption (tools/dbg_lanes2.py): two lanes (two ops.Ctx) sharing
read-only weights, each captured into its own graph, replayed concurrently.  DBG_CASE:
  lnet    models.LNet, two lanes of one module
  conv    a chain of 3x3 convs on one shared ConvW (two Ctx)
  modconv a chain of modulated convs on one shared ConvW (two Ctx)
  enet    models.ENet, two lanes of one module (the failing case)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import s2v_import  # noqa: E402,F401
from helpers import synth_sd  # noqa: E402
from s2v_amd import models, ops, synth  # noqa: E402
from s2v_amd.ops import NHWC, ConvW  # noqa: E402
from s2v_amd.runtime import GraphRunner  # noqa: E402

dev = "cuda"
CASE = os.environ.get("DBG_CASE", "conv")
REPS = int(os.environ.get("DBG_REPS", "4"))
B = 4
tag = " ".join(f"{k}={os.environ[k]}" for k in ("S2V_ENET_OVERLAP", "S2V_LNET_BRANCHES", "DBG_CASE", "S2V_PRECISION")
               if k in os.environ)


def inputs(seed, size=256):
    return [torch.from_numpy(a).to(dev) for a in synth.lipsync_inputs(f"lanes{seed}", B, size)]


def report(name, got, ref):
    out = []
    for i, (g, r) in enumerate(zip(got, ref)):
        d = (g - r).abs()
        nz = int((d != 0).sum())
        if nz:
            out.append(f"out{i}: {nz}/{d.numel()} differ, max {float(d.max()):.3e}")
    print(f"  [{tag}] {name}: {'OK' if not out else '; '.join(out)}", flush=True)


def make_runners():
    if CASE in ("lnet", "enet"):
        if CASE == "lnet":
            m = models.LNet()
            m.load_state_dict(synth_sd("lnet"))
        else:
            sd = {k: (torch.zeros_like(v) if k.startswith("style_convs.") and k.endswith(".weight") and v.numel() == 1
                      else v) for k, v in synth_sd("enet").items()}
            m = models.ENet()
            m.load_state_dict(sd)
        m.eval()
        rs = []
        for lane in range(2):
            x = inputs(lane)
            if CASE == "lnet":
                x = [x[0], F.interpolate(x[1], size=(96, 96), mode="bilinear", align_corners=False)]
            rs.append(GraphRunner(lambda *a, _l=lane: (m(*a, lane=_l),) if CASE == "lnet" else m(*a, lane=_l), x,
                                  warmup=1))
        return rs
    g = torch.Generator().manual_seed(0)
    cin = 256
    if CASE == "conv":
        h = 24
        cw = ConvW(torch.randn(cin, cin, 3, 3, generator=g) * 0.02, torch.randn(cin, generator=g) * 0.1, dev, padding=1)
    else:
        h = 100
        cw = ConvW(torch.randn(cin, cin, 3, 3, generator=g) * 0.02, torch.randn(cin, generator=g) * 0.1, dev, padding=1)
        wsq = torch.randn(cin, cin, 3, 3, generator=g).pow(2).sum((2, 3)).to(dev)
    rs = []
    for lane in range(2):
        ctx = ops.Ctx(dev)
        x0 = torch.rand((B, h, h, cin), generator=g).to(dev)

        def fwd(x, _ctx=ctx):
            cur = NHWC(x)
            for i in range(6):
                y = NHWC.empty(B, h, h, cin, dev)
                if CASE == "conv":
                    ops.conv2d(_ctx, cur, cw, y, act=ops.ACT_LRELU, alpha=0.2)
                else:
                    s = torch.full((B, cin), 0.5 + 0.1 * i, device=dev)
                    d = torch.empty((B, cin), device=dev)
                    ops.modconv_demod(_ctx, s, wsq, d, eps=1e-8, post=1.4142)
                    ops.modulated_conv2d(_ctx, cur, cw, y, s, d, act=ops.ACT_LRELU, alpha=0.2)
                cur = y
            return (cur.t,)
        rs.append(GraphRunner(fwd, [x0], warmup=1))
    return rs


runners = make_runners()
names = [f"lane{i}" for i in range(len(runners))]
seq = []
for r in runners:
    r.replay()
    torch.cuda.synchronize()
    seq.append(tuple(t.clone() for t in r.static_out))
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
