#!/usr/bin/env python3
"""Benchmark of the per-frame lip-sync hot path on MI355X (BASELINE.json metric).

Workload (one "step"): ENet(+LNet) forward — models/ENet.py:82-139 — on one batch of B=16
synthetic 256x256 face crops + 16 mel windows [1,80,16] (inference.py:393-399 batching,
LNet_batch_size 16), weights from the portable synthetic checkpoint (s2v_amd.synth), inputs
resident in HBM.  The whole forward is one HIP-graph replay.

Multi-GPU: one process per GPU (torchrun); frames shard across ranks with no data-path collective
(weak scaling: every rank runs its own B-frame batches); the timed region is bracketed by a barrier
and synchronize on every rank and the max over ranks is reported.

Prints ONE JSON line on rank 0 with the live roofline of the dominant kernel (HIP events on the
stream the kernels run on) and, at N=1, the CPU baseline (oracle restatement on host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import s2v_import  # noqa: E402,F401

METRIC = "synthesized 256×256 frames/sec/GPU (LNet+ENet path); 1/2/4/8-GPU scaling"
FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 matrix 157.3 TF (spec)
REF_GFLOP_PER_FRAME = 407.46       # ENet+LNet algorithmic GFLOP/frame (2*MAC)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    return ap.parse_args()


def make_inputs(batch, size, device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    mel = torch.rand((batch, 1, 80, 16), generator=g, device=device) * 8 - 4
    face = torch.rand((batch, 6, size, size), generator=g, device=device)
    face[:, :3, size // 2:] = 0.0                      # masked lower half (inference.py:397)
    gt = face[:, 3:].clone()
    return mel, face, gt


def live_roofline(model, inputs):
    """One un-graphed forward with every conv/GEMM launch bracketed by HIP events on its stream;
    per kernel symbol: sum of algorithmic FLOPs / sum of durations."""
    from s2v_amd import ops
    recs = []

    def hook(ctx, p, flops, launch):
        sym = ops.conv_symbol(ctx, p)
        splits = ops.conv_splits(ctx, p)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        recs.append((sym, flops, splits, s, e))

    ops.CONV_HOOK = hook
    try:
        with torch.no_grad():
            model(*inputs)
        torch.cuda.synchronize()
    finally:
        ops.CONV_HOOK = None
    per = {}
    for sym, flops, splits, s, e in recs:
        d = per.setdefault(sym, {"flops": 0.0, "ms": 0.0, "launches": 0, "split_launches": 0})
        d["flops"] += flops
        d["ms"] += s.elapsed_time(e)
        d["launches"] += 1
        d["split_launches"] += int(splits > 1)
    dom = max(per, key=lambda k: per[k]["ms"])
    if os.environ.get("S2V_BENCH_VERBOSE"):
        for k in sorted(per, key=lambda k: -per[k]["ms"]):
            v = per[k]
            tf = v["flops"] / max(v["ms"], 1e-9) / 1e9
            print(f"  {v['ms']:9.3f} ms  {v['launches']:4d} launches  {tf:7.2f} TF/s  {k}", file=sys.stderr)
    d = per[dom]
    achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
    total_ms = sum(v["ms"] for v in per.values())
    total_flops = sum(v["flops"] for v in per.values())
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_r01.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            traffic = json.load(f).get("per_launch_bytes", {}).get(dom)
    return {
        "bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
        "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
        "kernel": dom, "launches": d["launches"], "avg_launch_us": round(1e3 * d["ms"] / d["launches"], 2),
        "flops_per_launch": d["flops"] / d["launches"],
        "conv_family": {"achieved": round(total_flops / (total_ms * 1e-3) / 1e12, 2),
                        "ms_per_step": round(total_ms, 3), "symbols": len(per)},
    }


def cpu_baseline(sd, batch, size, threads, seconds):
    """Oracle (CPU restatement, oracle/nets.py) on the host cores, bounded sample."""
    from oracle import nets
    torch.set_num_threads(threads)
    mel, face, gt = make_inputs(batch, size, "cpu", 1234)
    frames, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            nets.enet_forward(sd, mel, face, gt)
            frames += batch
            el = time.perf_counter() - t0
            if el >= seconds or frames >= 8 * batch:
                break
    return {"value": round(frames / el, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{frames} frames ({batch}-frame batches) of the same ENet(+LNet) {size}x{size} workload "
                      f"in {el:.1f}s, torch CPU fp32, {threads} threads"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    from s2v_amd import models, synth
    from s2v_amd.models import arch
    from s2v_amd.runtime import GraphRunner

    sd = synth.synth_torch_state_dict(arch.ENetParams(lnet=arch.LNetParams()))
    model = models.ENet()
    model.load_state_dict(sd)
    model.eval()
    inputs = make_inputs(args.batch, args.size, dev, 1000 + rank)
    fn = lambda m, f, g: model(m, f, g)  # noqa: E731
    if args.no_graph:
        step = lambda: fn(*inputs)  # noqa: E731
        for _ in range(max(1, args.warmup)):
            step()
    else:
        runner = GraphRunner(fn, list(inputs), warmup=1)
        step = runner.replay
        for _ in range(args.warmup):
            step()

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    frames = world * args.batch * args.steps
    value = frames / elapsed
    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"ENet(+LNet) forward, B={args.batch} synthetic {args.size}x{args.size} crops "
                               f"+ [1,80,16] mel windows -> 384x384 (models/ENet.py:82-139)",
                   "global_batch": world * args.batch, "batch_per_gpu": args.batch, "crop": args.size,
                   "parallelism": f"frame-shard x{world} (no data-path collective)",
                   "graph": not args.no_graph,
                   "achieved_tflops_algorithmic": round(value * REF_GFLOP_PER_FRAME / 1e3, 2)},
    }
    if rank == 0 and not args.no_roofline:
        result["roofline"] = live_roofline(model, inputs)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        result["cpu_baseline"] = cpu_baseline(sd, 2, args.size, threads, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
