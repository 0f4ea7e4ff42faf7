#!/usr/bin/env python3
"""Kernel symbols (and conv keys) of every conv launch of one eager forward of a bench workload:
python tools/plan_syms.py lipsync [--match halo]"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    sys.argv = [sys.argv[0]]
    bargs = bench.parse()
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[a.workload](bargs, dev, 0, 1)
    seen = collections.Counter()

    def hook(ctx, p, flops, launch):
        sym = ops.plan_symbol(p.plan)
        if a.match in sym:
            seen[(sym, f"n{p.n} {p.h}x{p.w}x{p.cin} -> {p.oh}x{p.ow}x{p.cout} k{p.kh}x{p.kw}")] += 1
        launch()
    with torch.no_grad():
        wl.forward()
        torch.cuda.synchronize()
        ops.CONV_HOOK = hook
        try:
            wl.forward()
        finally:
            ops.CONV_HOOK = None
        torch.cuda.synchronize()
    for (sym, shape), c in sorted(seen.items(), key=lambda kv: -kv[1]):
        print(f"{c:4d}  {sym[10:60]:50s} {shape}")


if __name__ == "__main__":
    main()
