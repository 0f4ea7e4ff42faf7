#!/usr/bin/env python3
"""Time every split-precision tile (force_tile 1..8) of the implicit-GEMM conv on the model's
representative shapes (HIP events, f16x3 by default) — the data behind conv.hip's kX3Tiles rates.

    python tools/tile_sweep.py [--prec f16x3] [--iters 10]
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

SHAPES = [  # (name, n, h, w, cin, cout, k, stride)
    ("enet 256^2 256->256", 16, 256, 256, 256, 256, 3, 1),
    ("styleconv 400^2 256->128", 16, 400, 400, 256, 128, 3, 1),
    ("styleconv 400^2 128->128", 16, 400, 400, 128, 128, 3, 1),
    ("enet 64^2 512->512", 16, 64, 64, 512, 512, 3, 1),
    ("enet 32^2 512->512", 16, 32, 32, 512, 512, 3, 1),
    ("lnet 12^2 1024->256", 16, 12, 12, 1024, 256, 3, 1),
    ("lnet 12^2 256->768", 16, 12, 12, 256, 768, 3, 1),
    ("lnet 24^2 256->512", 16, 24, 24, 256, 512, 3, 1),
    ("lnet 48^2 128->128", 16, 48, 48, 128, 128, 3, 1),
    ("lnet 96^2 64->64", 16, 96, 96, 64, 64, 3, 1),
    ("dnet 64^2 256->256", 16, 64, 64, 256, 256, 3, 1),
    ("dnet 128^2 128->128", 16, 128, 128, 128, 128, 3, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="f16x3")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    ops.set_precision(a.prec)
    dev = torch.device("cuda")
    ctx = ops.Ctx(dev)
    for name, n, h, w, cin, cout, k, st in SHAPES:
        wt = torch.randn(cout, cin, k, k) / math.sqrt(cin * k * k)
        cw = ConvW(wt, torch.randn(cout), dev, stride=st, padding=k // 2)
        x = NHWC(torch.randn(n, h, w, cin, device=dev))
        oh, ow = cw.out_hw(h, w)
        y = NHWC.empty(n, oh, ow, cout, dev)
        flops = 2.0 * n * oh * ow * k * k * cin * cout
        row = []
        for t in [0] + list(range(1, 10)):
            try:
                ops.conv2d(ctx, x, cw, y, force_tile=t)
            except Exception:        # tile not offered for this shape (weight rows past npad)
                row.append(f"t{t}:  -  ")
                continue
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                ops.conv2d(ctx, x, cw, y, force_tile=t)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.iters
            row.append(f"t{t}:{flops / ms / 1e9:6.1f}")
        print(f"{name:28s} " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
