#!/usr/bin/env python3
"""Time every conv shape of one LNet decoder FFC block at B=16 (default plan, forced split-K and
tiles), to see where LNet's conv time goes.   python tools/lnet_convs.py [--iters 50]"""
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

# (name, h, w, cin, cout, k, reflect) per level: 12^2 c=1024, 24^2 c=256, 48^2 c=128 (LNet.py:46-77)
SHAPES = []
for h, c in ((12, 1024), (24, 256), (48, 128)):
    cg = int(c * 0.75)
    cl, cc = c - cg, cg // 2
    f = h * (h // 2 + 1)
    SHAPES += [(f"{h}:to_l", h, h, c, cl, 3, True), (f"{h}:l2g", h, h, cl, cg, 3, True),
               (f"{h}:st1", h, h, cg, cc, 1, False), (f"{h}:fu", f, 1, 2 * cc, 2 * cc, 1, False),
               (f"{h}:st2", h, h, cc, cg, 1, False)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--splits", default="0,1,2,4,8")
    ap.add_argument("--tiles", default="0")
    ap.add_argument("--only", default="", help="comma list of shape names")
    ap.add_argument("--pad", default="reflect", choices=("reflect", "zero", "valid"),
                    help="3x3 convs: reflect padding (the model), zero padding, or a pre-padded (h+2) input")
    ap.add_argument("--graph", action="store_true", help="time the launches as one captured HIP graph")
    ap.add_argument("--prec", default="f16x3")
    a = ap.parse_args()
    ops.set_precision(a.prec)
    dev = torch.device("cuda")
    ctx = ops.Ctx(dev)
    total = {}
    for name, h, w, cin, cout, k, refl in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        wt = torch.randn(cout, cin, k, k) / math.sqrt(cin * k * k)
        valid = refl and a.pad == "valid"
        mode = ops.PAD_REFLECT if (refl and a.pad == "reflect") else ops.PAD_ZERO
        cw = ConvW(wt, torch.randn(cout), dev, padding=0 if valid else k // 2, pad_mode=mode)
        x = NHWC(torch.randn(a.n, h + 2 * valid, w + 2 * valid, cin, device=dev))
        y = NHWC.empty(a.n, h, w, cout, dev)
        flops = 2.0 * a.n * h * w * k * k * cin * cout
        res = []
        for t in [int(v) for v in a.tiles.split(",")]:
            for sp in [int(v) for v in a.splits.split(",")]:
                kw = dict(force_tile=t, force_splits=sp)
                try:
                    ops.conv2d(ctx, x, cw, y, **kw)
                except Exception as e:  # noqa: BLE001
                    res.append(f"t{t}s{sp}: -")
                    continue
                torch.cuda.synchronize()
                g = None
                if a.graph:
                    st = torch.cuda.Stream()
                    st.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(st):
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, stream=st):
                            for _ in range(a.iters):
                                ops.conv2d(ctx, x, cw, y, **kw)
                    torch.cuda.current_stream().wait_stream(st)
                    g.replay()
                    torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                if g is not None:
                    g.replay()
                else:
                    for _ in range(a.iters):
                        ops.conv2d(ctx, x, cw, y, **kw)
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) * 1e3 / a.iters
                res.append(f"t{t}s{sp}:{us:6.1f}us {flops / us / 1e6:5.0f}TF")
                if t == 0 and sp == 0:
                    total[name] = us
                    p = ops._lib.ConvParams()
        print(f"{name:10s} M={a.n * h * w:6d} K={k * k * cin:5d} N={cout:4d} {flops / 1e9:6.2f}GF  " + "  ".join(res),
              flush=True)
    print("default plan, one FFC (x18 per level):", {k: round(v, 1) for k, v in total.items()})
    for h in (12, 24, 48):
        print(f"level {h}: {sum(v for k, v in total.items() if k.startswith(f'{h}:')) * 18 / 1e3:.2f} ms per forward")


if __name__ == "__main__":
    main()
