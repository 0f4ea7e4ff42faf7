#!/usr/bin/env python3
"""Graph-timed micro-benchmark of LNet's fused FFC kernels (csrc/ffc.hip) against the separate launches
they replace, one FineADAINLama per decoder level at B = 16, each kernel alone and back to back.

    python tools/ffc_micro.py [--iters 20] [--prec f16x3]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402
from s2v_amd.ops import NHWC  # noqa: E402


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
    best = 1e30
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) * 1e3 / n)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--prec", default="f16x3")
    ap.add_argument("--b", type=int, default=16)
    a = ap.parse_args()
    from helpers import synth_sd
    from s2v_amd.engine import lnet
    dev = torch.device("cuda")
    ops.set_precision(a.prec)
    eng = lnet.LNetEngine(synth_sd("lnet"), dev)
    ctx = ops.Ctx(dev)
    b = a.b
    for lv in eng.levels:
        f1 = lv["blocks"][0][0]
        h, c, cl, cg, cc = f1.h, f1.c, f1.cl, f1.cg, f1.cc
        x = NHWC(torch.randn(b, h, h, c, device=dev))
        y = NHWC(torch.randn(b, h, h, c, device=dev))
        out = NHWC.empty(b, h, h, c, dev)
        t1 = NHWC.empty(b, h, h, cc, dev)
        spec = torch.empty((b, f1.F, 2 * cc), device=dev)
        spec2 = NHWC.empty(b, f1.F, 1, 2 * cc, dev)
        u = NHWC.empty(b, h, h, cc, dev)
        g = torch.zeros((b, c), device=dev)
        xg = x.slice(cl, cg)
        res = {
            "spec_fwd": lambda: ops.ffc_spec_fwd(ctx, xg, f1.st1, f1.fft, t1, spec),
            "spec_inv": lambda: ops.ffc_spec_inv(ctx, spec, f1.fu, f1.fft, t1, u),
            "norm": lambda: ops.ffc_norm(ctx, y, u, f1.st2, out, g, g, act=ops.ACT_LRELU, alpha=0.01),
            "st1": lambda: ops.conv2d(ctx, xg, f1.st1, t1, act=ops.ACT_RELU, force_splits=1),
            "rfft2": lambda: ops.rfft2(ctx, t1, f1.fft, spec),
            "fu": lambda: ops.conv2d(ctx, NHWC(spec.view(b, f1.F, 1, 2 * cc)), f1.fu, spec2, act=ops.ACT_RELU,
                                     force_splits=1),
            "irfft2": lambda: ops.irfft2(ctx, spec2.t.view(b, f1.F, 2 * cc), f1.fft, u, res=t1),
            "st2": lambda: ops.conv2d(ctx, u, f1.st2, y.slice(cl, cg), res=y.slice(cl, cg), force_splits=1),
            "instnorm": lambda: ops.instnorm(ctx, y, out, g, g, act=ops.ACT_LRELU, alpha=0.01),
        }
        line = []
        for k, fn in res.items():
            fn()
            torch.cuda.synchronize()
            line.append(f"{k} {graph_us(fn, a.iters):6.1f}")
        fused = sum(float(v.split()[1]) for v in line[:3])
        sep = sum(float(v.split()[1]) for v in line[3:])
        print(f"h={h:2d} B={b}: " + "  ".join(line) + f"   | fused {fused:.1f} vs separate {sep:.1f} us", flush=True)


if __name__ == "__main__":
    main()
