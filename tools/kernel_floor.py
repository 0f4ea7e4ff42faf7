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
    a = ap.parse_args()
    dev = torch.device("cuda")
    ctx = ops.Ctx(dev)
    t = torch.empty(256, device=dev)
    print(f"fill 256 floats: {graph_us(lambda: ops.fill(ctx, t, 1.0), a.n):.2f} us per dependent launch", flush=True)
    big = torch.empty(1 << 24, device=dev)
    print(f"fill 64 MB: {graph_us(lambda: ops.fill(ctx, big, 1.0), 20):.2f} us per launch", flush=True)
    cw = ConvW(torch.randn(64, 32, 1, 1) / 6, None, dev)
    x = NHWC(torch.randn(1, 8, 8, 32, device=dev))
    y = NHWC.empty(1, 8, 8, 64, dev)
    for prec in ("f16x3",):
        ops.set_precision(prec)
        us = graph_us(lambda: ops.conv2d(ctx, x, cw, y), a.n)
        print(f"1x1 conv 64 px x 32 -> 64 ({prec}, one 64x64 block, one K slice): {us:.2f} us per dependent launch",
              flush=True)


if __name__ == "__main__":
    main()
