#!/usr/bin/env python3
"""Micro-benchmark of one libs2v convolution shape (for kernel tuning and PMC passes).

    python tools/conv_micro.py --n 16 --h 200 --w 200 --cin 256 --cout 128 --k 3 [--up2] [--iters 20]

Prints the launch plan, the average time (HIP events on the launch stream) and the algorithmic
TFLOP/s.  ``--sweep`` times every tile config the kernel offers for the shape.
"""
import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402
from s2v_amd.ops import NHWC, ConvW  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--h", type=int, default=200)
    ap.add_argument("--w", type=int, default=200)
    ap.add_argument("--cin", type=int, default=256)
    ap.add_argument("--cout", type=int, default=128)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--pad", type=int, default=-1, help="padding (default k // 2)")
    ap.add_argument("--up2", action="store_true", help="nearest-x2 upsampled input (IN_NEAREST_UP2)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--splits", default="0", help="comma list of force_splits values")
    ap.add_argument("--prec", default="both", choices=("f32", "bf16x3", "f16x3", "both", "split"))
    ap.add_argument("--tiles", default="", help="comma list of force_tile values (101.. = x3 variants)")
    ap.add_argument("--glds", action="store_true", help="also time the LDS-DMA kernel on a split-layout input")
    ap.add_argument("--graph", action="store_true",
                    help="time the launches as one captured HIP graph (no host launch overhead in the timing)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    ctx = ops.Ctx(dev)
    w = torch.randn(a.cout, a.cin, a.k, a.k) / math.sqrt(a.cin * a.k * a.k)
    cw = ConvW(w, torch.randn(a.cout), dev, stride=a.stride, padding=a.k // 2 if a.pad < 0 else a.pad,
               in_mode=ops.IN_NEAREST_UP2 if a.up2 else ops.IN_DIRECT)
    x = NHWC(torch.randn(a.n, a.h, a.w, a.cin, device=dev))
    oh, ow = cw.out_hw(a.h, a.w)
    y = NHWC.empty(a.n, oh, ow, a.cout, dev)
    flops = 2.0 * a.n * oh * ow * a.k * a.k * a.cin * a.cout
    tiles = [int(t) for t in a.tiles.split(",")] if a.tiles else (range(1, 7) if a.sweep else [0])
    precs = {"both": ("f32", "f16x3"), "split": ("bf16x3", "f16x3")}.get(a.prec, (a.prec,))
    splits_list = [int(v) for v in a.splits.split(",")]
    a.splits = splits_list[0]
    ref = {}
    for prec, t, sp in [(p, t, sp) for p in precs for t in tiles for sp in splits_list
                        if not (t > 100 and p == "f32")]:
        ops.set_precision(prec)
        if prec not in ref:                   # the planner's launch: reference output of this precision
            ops.conv2d(ctx, x, cw, y, act=ops.ACT_LRELU, alpha=0.2)
            ref[prec] = y.t.clone()
        kw = dict(act=ops.ACT_LRELU, alpha=0.2, force_tile=t, force_splits=sp)
        try:
            ops.conv2d(ctx, x, cw, y, **kw)
        except Exception as ex:  # noqa: BLE001
            print(f"tile={t} splits={sp}: {ex}", flush=True)
            continue
        torch.cuda.synchronize()
        md = (y.t - ref[prec]).abs().max().item() / max(ref[prec].abs().max().item(), 1e-30)
        ms = _time(lambda: ops.conv2d(ctx, x, cw, y, **kw), a.iters, a.graph)
        pp = _params(ctx, x, cw, y, t, sp)
        print(f"tile={t} splits={ops.conv_splits(ctx, pp)} {ops.conv_symbol(ctx, pp)}: {ms * 1e3:9.1f} us  "
              f"{flops / ms / 1e9:7.2f} TFLOP/s  rel.diff vs planner {md:.2e}", flush=True)
    if a.glds and not a.up2 and a.stride == 1:
        ops.set_precision("f16x3")
        xs = ops.split_act(ctx, x)
        y2 = NHWC.empty(a.n, oh, ow, a.cout, dev)
        kw = dict(act=ops.ACT_LRELU, alpha=0.2, force_splits=a.splits)
        ops.conv2d(ctx, x, cw, y, **kw)
        ops.conv2d(ctx, xs, cw, y2, **kw)
        torch.cuda.synchronize()
        same = bool(torch.equal(y.t, y2.t))
        md = (y.t - y2.t).abs().max().item()
        for name, fn in (("split_act", lambda: ops.split_act(ctx, x, xs)),
                         ("glds conv", lambda: ops.conv2d(ctx, xs, cw, y2, **kw))):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.iters
            extra = f"{flops / ms / 1e9:7.2f} TFLOP/s  bitwise={same} maxdiff={md:.3g}" if name == "glds conv" else \
                f"{x.t.numel() * 8 / ms / 1e9:7.1f} GB/s"
            print(f"{name} {ops.conv_symbol(ctx, _params(ctx, xs, cw, y2, 0, a.splits)) if name == 'glds conv' else ''}: "
                  f"{ms * 1e3:9.1f} us  {extra}", flush=True)


def _time(fn, iters, graph):
    """Average ms per call of ``fn`` over ``iters`` back-to-back calls (HIP events); with ``graph`` the
    calls are captured once into a HIP graph and the replay is timed (device time only)."""
    if graph:
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            fn()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=st):
                for _ in range(iters):
                    fn()
        torch.cuda.current_stream().wait_stream(st)
        g.replay()
        torch.cuda.synchronize()
        run = g.replay
        reps = 1
    else:
        run = fn
        reps = iters
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def _params(ctx, x, cw, y, tile, splits):
    captured = {}

    def hook(c, p, flops, launch):
        captured["p"] = p
    ops.CONV_HOOK = hook
    try:
        ops.conv2d(ctx, x, cw, y, force_tile=tile, force_splits=splits)
    finally:
        ops.CONV_HOOK = None
    return captured["p"]


if __name__ == "__main__":
    main()
