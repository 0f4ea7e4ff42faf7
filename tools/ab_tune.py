#!/usr/bin/env python3
"""A/B a planner knob (s2v_tune) on one bench workload inside ONE process: the graph-replayed step
is re-captured per setting and the settings are timed alternately, so box-to-box noise cancels.

    python tools/ab_tune.py --workload lipsync --key 3 --values 0,360 --rounds 4 --steps 10
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import s2v_import  # noqa: E402,F401
from s2v_amd import ops  # noqa: E402
from s2v_amd.runtime import GraphRunner  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="lipsync")
    ap.add_argument("--key", type=int, required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    sys.argv = [sys.argv[0], "--workload", a.workload]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = bench.WORKLOADS[a.workload](args, dev, 0, 1)
    ctx = ops.Ctx(dev)
    vals = [int(v) for v in a.values.split(",")]
    runners = {}
    for v in vals:
        ops.tune(ctx, a.key, v)
        runners[v] = GraphRunner(wl.fn, list(wl.inputs), warmup=1)
    res = {v: [] for v in vals}
    for _ in range(a.rounds):
        for v in vals:
            r = runners[v]
            r.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                r.replay()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / a.steps * 1e3)
    for v in vals:
        ms = sorted(res[v])
        print(f"key {a.key} = {v}: ms/step min {ms[0]:.3f} median {ms[len(ms) // 2]:.3f}  "
              f"({wl.batch / ms[0] * 1e3:.1f} units/s at the min)", flush=True)


if __name__ == "__main__":
    main()
