#!/usr/bin/env python3
"""Debug: memory written by both lanes' captured graphs.  Every s2v op called while capturing lane
L's ENet forward logs its tensor arguments (storage range, written or read per the op schema);
overlapping ranges between the two lanes where either side writes are printed (tools/dbg_lanes4.py
found the divergence; this names the shared buffer)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from helpers import synth_sd  # noqa: E402
from s2v_amd import models, ops, synth, torch_ops  # noqa: E402
from s2v_amd.runtime import GraphRunner  # noqa: E402

dev = "cuda"
B = 4
LOG = {}
KEEP = {}      # lane -> {(start, end): storage}: kept alive so they can be snapshotted (no intra-graph reuse)
CUR = [None]
CUR_LANE = [None]


class Logged:
    def __getattr__(self, name):
        op = getattr(torch_ops.load(), name)
        schema = op.default._schema if hasattr(op, "default") else None

        def call(*a, **k):
            if CUR[0] is not None and schema is not None:
                for i, (arg, v) in enumerate(zip(schema.arguments, a)):
                    if isinstance(v, torch.Tensor) and v.is_cuda:
                        st = v.untyped_storage()
                        w = arg.alias_info is not None and arg.alias_info.is_write
                        CUR[0].append((st.data_ptr(), st.data_ptr() + st.nbytes(), w, f"{name}.{arg.name}",
                                       tuple(v.shape)))
                        KEEP[CUR_LANE[0]][(st.data_ptr(), st.data_ptr() + st.nbytes())] = st
            return op(*a, **k)
        return call


ops.S2V = Logged()

sd = {k: (torch.zeros_like(v) if k.startswith("style_convs.") and k.endswith(".weight") and v.numel() == 1
          else v) for k, v in synth_sd("enet").items()}
m = models.ENet()
m.load_state_dict(sd)
m.eval()


class Probe(GraphRunner):
    def __init__(self, lane, x):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            m(*x, lane=lane)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.static_in = [t.clone() for t in x]
        self.graph = torch.cuda.CUDAGraph()
        LOG[lane] = []
        KEEP[lane] = {}
        CUR_LANE[0] = lane
        CUR[0] = LOG[lane]
        with torch.cuda.graph(self.graph):
            self.static_out = m(*self.static_in, lane=lane)
        CUR[0] = None
        torch.cuda.synchronize()


rs = [Probe(lane, [torch.from_numpy(a).to(dev) for a in synth.lipsync_inputs(f"lanes{lane}", B, 256)])
      for lane in range(2)]
print({k: len(v) for k, v in LOG.items()}, "tensor args logged per lane", flush=True)




def storages(lane):
    """unique (start, end) -> names of the lane's s2v op tensor storages"""
    d = {}
    for a, b, w, n, shp in LOG[lane]:
        d.setdefault((a, b), set()).add(n + ("!" if w else ""))
    return d


def u8(st):
    return torch.empty(0, dtype=torch.uint8, device=dev).set_(st)


shared = set(storages(0)) & set(storages(1))
for victim, other in ((0, 1), (1, 0)):
    rs[victim].graph.replay()
    torch.cuda.synchronize()
    names = storages(victim)
    priv = {k: st for k, st in KEEP[victim].items() if k not in shared}
    before = {k: u8(st).clone() for k, st in priv.items()}
    rs[other].graph.replay()
    torch.cuda.synchronize()
    changed = [(k, int((u8(priv[k]) != before[k]).sum())) for k in priv if not torch.equal(u8(priv[k]), before[k])]
    print(f"victim lane {victim}: {len(priv)} private storages ({sum(b - a for a, b in priv) / 1e6:.1f} MB); "
          f"changed by lane {other}'s replay: {len(changed)}", flush=True)
    for (a, b), nb in changed[:20]:
        print(f"   [{a:#x}, {b:#x}) {nb} bytes changed; used as {sorted(names[(a, b)])[:6]}", flush=True)
hits = {}
for a0, b0, w0, n0, s0 in LOG[0]:
    for a1, b1, w1, n1, s1 in LOG[1]:
        if a0 < b1 and a1 < b0 and (w0 or w1):
            key = (n0, s0, w0, n1, s1, w1, a0 == a1)
            hits[key] = hits.get(key, 0) + 1
print(f"{len(hits)} overlapping (op.arg, shape, written) pairs between the lanes:")
for k, c in sorted(hits.items(), key=lambda kv: -kv[1])[:40]:
    n0, s0, w0, n1, s1, w1, same = k
    print(f"  x{c}: lane0 {n0}{list(s0)} {'W' if w0 else 'R'}  <->  lane1 {n1}{list(s1)} {'W' if w1 else 'R'}"
          f"{'  (same storage)' if same else ''}")
