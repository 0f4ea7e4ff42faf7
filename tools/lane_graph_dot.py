#!/usr/bin/env python3
"""Dump the captured ENet(+LNet) lane graphs (hipGraphDebugDotPrint via torch.cuda.CUDAGraph.debug_dump)
and check the dependency edges of every x2 bilinear upsample node (the r03 cross-lane
corruption): each up2 / resize kernel node must depend on the kernel captured right before it on its
stream — the producer of its input in every use of the kernel in the model — through a path of edges.

    python tools/lane_graph_dot.py --out gpurun_out/graph [--lanes 2] [--batch 4]

Writes <out>/lane<i>.dot and prints, per lane, the kernel-node count, edge count and the up2 nodes
with their parents; exits 1 when an up2 node is not reachable from its capture-order predecessor on
the same stream (a missing edge)."""
import argparse
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401


def parse_dot(path):
    """hipGraphDebugDotPrint output: multi-line record nodes ``"graph_0_node_N"[... label="{ KERNEL | {ID | N |
    symbol\\<\\<\\<grid...`` and edges ``"a" -> "b"``; returns ({node: "KIND symbol"}, [(src, dst)])."""
    text = open(path).read()
    nodes = {}
    for m in re.finditer(r'"(\w+)"\[[^\n]*label="\{\s*\n?(\w+)\s*\n?\|\s*\{ID \| \d+ \| ([^\\|<]*)', text):
        nodes[m.group(1)] = f"{m.group(2)} {m.group(3).strip()}"
    edges = re.findall(r'"(\w+)"\s*->\s*"(\w+)"', text)
    return nodes, edges


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/graph")
    ap.add_argument("--lanes", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    from s2v_amd import models, synth
    from s2v_amd.models import arch
    dev = torch.device("cuda")
    sd = synth.synth_torch_state_dict(arch.ENetParams(lnet=arch.LNetParams()))
    model = models.ENet()
    model.load_state_dict(sd)
    model.eval()
    g = torch.Generator(device=dev).manual_seed(3)
    mel = torch.rand((a.batch, 1, 80, 16), generator=g, device=dev)
    face = torch.rand((a.batch, 6, 256, 256), generator=g, device=dev)
    gt = face[:, 3:].clone()
    bad = 0
    for lane in range(a.lanes):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            model(mel, face, gt, lane=lane)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        cg = torch.cuda.CUDAGraph(keep_graph=True)     # the captured graph object survives capture_end
        cg.enable_debug_mode()
        with torch.cuda.graph(cg):
            model(mel, face, gt, lane=lane)
        torch.cuda.synchronize()
        path = os.path.join(a.out, f"lane{lane}.dot")
        cg.debug_dump(path)
        if not os.path.exists(path):
            sys.exit(f"debug_dump wrote nothing to {path}")
        bad += check(lane, path)
    sys.exit(1 if bad else 0)


def check(lane, path):
    """Edge check of one dumped lane graph; returns the number of up2 / resize nodes that have no path
    from any of their six capture-order predecessors."""
    nodes, edges = parse_dot(path)
    parents = {}
    for s, d in edges:
        parents.setdefault(d, set()).add(s)
    order = sorted(nodes, key=lambda k: int(re.sub(r"\D", "", k.rsplit("_", 1)[-1]) or 0))
    kern = [k for k in order if nodes[k].startswith("KERNEL")]
    up = [k for k in kern if "up2_bilinear" in nodes[k] or "resize" in nodes[k]]

    def ancestors(k):
        seen, st = set(), [k]
        while st:
            for p in parents.get(st.pop(), ()):
                if p not in seen:
                    seen.add(p)
                    st.append(p)
        return seen
    roots = [k for k in nodes if k not in parents]
    print(f"lane {lane}: {len(nodes)} nodes ({len(kern)} kernels), {len(edges)} edges, {len(roots)} roots, "
          f"{len(up)} resize / up2 nodes", flush=True)
    bad = 0
    for k in up:
        i = kern.index(k)
        anc = ancestors(k)
        prev = kern[max(0, i - 6):i]
        linked = [p for p in prev if p in anc]
        ok = bool(linked) or i == 0
        bad += not ok
        print(f"  {k}: {nodes[k][7:80]!r} parents={sorted(parents.get(k, ()))} ancestors={len(anc)} "
              f"linked-prev={linked[-2:]} {'OK' if ok else 'NO PATH FROM ITS PREDECESSORS'}", flush=True)
    return bad


def parse_only(paths):
    """Check already dumped .dot files (no GPU)."""
    sys.exit(1 if sum(check(i, p) for i, p in enumerate(paths)) else 0)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--check":
        parse_only(sys.argv[2:])
    main()
