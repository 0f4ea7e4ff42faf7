#!/usr/bin/env python3
"""Debug: standalone reproducer of the lane divergence found by tools/dbg_lanes4.py (the first
differing tensor is always an up2_bilinear_nhwc4_kernel output: lanes 48-63 of a wave, odd dwords).
Two graphs of a resize chain (x2 bilinear up, generic x0.5 down, ...) replayed concurrently on two
streams; every up2 output is probed.  DBG_MODE: s2v (our kernels) | torch (F.interpolate only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402
from s2v_amd.ops import NHWC  # noqa: E402

dev = "cuda"
MODE = os.environ.get("DBG_MODE", "s2v")
C = int(os.environ.get("DBG_C", "4"))
H = int(os.environ.get("DBG_H", "200"))
N = int(os.environ.get("DBG_N", "4"))
STEPS = int(os.environ.get("DBG_STEPS", "20"))
REPS = int(os.environ.get("DBG_REPS", "10"))


def build(seed):
    ctx = ops.Ctx(dev)
    g = torch.Generator(device=dev).manual_seed(seed)
    x0 = torch.rand((N, H, H, C), generator=g, device=dev)
    probes = []

    def fwd():
        cur = x0
        for i in range(STEPS):
            if MODE == "s2v":
                up = NHWC.empty(N, 2 * H, 2 * H, C, dev)
                ops.resize_nhwc(ctx, NHWC(cur), up, scale_factor=2)
                probes.append(up.t.clone())
                dn = NHWC.empty(N, H, H, C, dev)
                ops.resize_nhwc(ctx, up, dn, scale_factor=0.5)
                cur = dn.t
            else:
                up = F.interpolate(cur.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear", align_corners=False)
                probes.append(up.clone())
                cur = F.interpolate(up, scale_factor=0.5, mode="bilinear", align_corners=False).permute(0, 2, 3, 1)
                cur = cur.contiguous()
        return cur
    fwd()
    torch.cuda.synchronize()
    probes.clear()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        fwd()
    torch.cuda.synchronize()
    return graph, probes, x0, ctx      # x0 / ctx: alive as long as the graph (it reads them)


runs = [build(1), build(2)]
seq = []
for g, p, *_ in runs:
    g.replay()
    torch.cuda.synchronize()
    seq.append([t.clone() for t in p])
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
cur = torch.cuda.current_stream()
bad = 0
for rep in range(REPS):
    for st in streams:
        st.wait_stream(cur)
    for (g, *_), st in zip(runs, streams):
        with torch.cuda.stream(st):
            g.replay()
    for st in streams:
        cur.wait_stream(st)
    torch.cuda.synchronize()
    for li, ((g, p, *_), s) in enumerate(zip(runs, seq)):
        for i, (a, b) in enumerate(zip(p, s)):
            if not torch.equal(a, b):
                nz = (a != b).nonzero()
                bad += 1
                print(f"  rep {rep} lane {li} probe {i}: {nz.shape[0]} differ, first {nz[:3].tolist()}", flush=True)
                break
print(f"[{MODE} C={C} H={H} N={N}] bad {bad} / {2 * REPS}", flush=True)
