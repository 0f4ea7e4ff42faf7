#!/usr/bin/env python3
"""Fixed cost of one dependent kernel launch in a HIP graph on this device: N tiny launches of a
trivial libs2v kernel (s2v::fill_value_ on 256 floats) captured back to back on one stream, and the
same for a 1-slice split-precision conv (64x64 tile), graph-timed.

    python tools/kernel_floor.py [--n 200]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402
from s2v_amd.ops import NHWC, ConvW  # noqa: E402


def graph_us(fn, n):
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / (5 * n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=200)
    ap.add_argument("--case", type=int, default=-1, help="run only conv case i (PMC passes)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    ctx = ops.Ctx(dev)
    t = torch.empty(256, device=dev)
    print(f"fill 256 floats: {graph_us(lambda: ops.fill(ctx, t, 1.0), a.n):.2f} us per dependent launch", flush=True)
    big = torch.empty(1 << 24, device=dev)
    print(f"fill 64 MB: {graph_us(lambda: ops.fill(ctx, big, 1.0), 20):.2f} us per launch", flush=True)
    ops.set_precision("f16x3")
    # 1x1 convs on the 64x64 tile (force_tile 5, no split-K): fixed cost per launch (1 block, 1 K-slice), the
    # cost per K-slice, and the dependence on the block count (LNet's FourierUnit / st1 / st2 shapes)
    cases = ((64, 32, 64), (64, 192, 64), (64, 768, 64), (4992, 32, 192), (4992, 192, 192),
             (4992, 768, 192), (36864, 32, 96), (36864, 96, 96), (2304, 768, 384))
    for i, (m, cin, cout) in enumerate(cases):
        if a.case >= 0 and i != a.case:
            continue
        cw = ConvW(torch.randn(cout, cin, 1, 1) / cin ** 0.5, None, dev)
        x = NHWC(torch.randn(1, m, 1, cin, device=dev))
        y = NHWC.empty(1, m, 1, cout, dev)
        ops.conv2d(ctx, x, cw, y, force_tile=5, force_splits=1)
        us = graph_us(lambda: ops.conv2d(ctx, x, cw, y, force_tile=5, force_splits=1), a.n)
        blocks = -(-m // 64) * -(-cout // 64)
        print(f"1x1 conv M={m:6d} K={cin:4d} N={cout:4d} 64x64 tile ({blocks:5d} blocks, {cin // 32:3d} K-slices): "
              f"{us:7.2f} us per dependent launch", flush=True)
        # the same conv alternating with a tiny fill (a different kernel between two conv launches)
        us2 = graph_us(lambda: (ops.fill(ctx, t, 1.0), ops.conv2d(ctx, x, cw, y, force_tile=5, force_splits=1)), a.n // 2)
        print(f"    alternating with fill: {us2:7.2f} us per (fill + conv)", flush=True)


if __name__ == "__main__":
    main()
