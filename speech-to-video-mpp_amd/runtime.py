"""HIP-graph capture of a whole forward (one launch-bound pass of ~1e3 kernels -> one graph
replay), the MI355X replacement for a tracing compiler, and lanes of captured forwards replayed
concurrently on their own streams."""
from __future__ import annotations

import torch


class GraphRunner:
    """Captures ``fn(*inputs)`` for fixed shapes.  Eager warm-up runs on a side stream first so the
    op workspaces and the caching allocator reach steady state before capture."""

    def __init__(self, fn, example_inputs, warmup: int = 2):
        self.fn = fn
        self.static_in = [t.clone() for t in example_inputs]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                fn(*self.static_in)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_out = fn(*self.static_in)
        torch.cuda.synchronize()

    def __call__(self, *inputs):
        for dst, src in zip(self.static_in, inputs):
            if src is not None and src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out

    def replay(self):
        self.graph.replay()
        return self.static_out


class LaneRunner:
    """``lanes`` captured graphs of ``fn(lane, *inputs)``, each with its own static inputs, outputs
    and execution lane (the model's per-lane ``ops.Ctx``: workspace, side streams, noise counters),
    replayed round-robin, each lane on a stream of its own.

    Successive steps therefore overlap: while lane 0 runs the MFMA-bound tail of its forward (ENet's
    StyleConv decoder), lane 1 runs the latency-bound head of the next batch (LNet's ~800-kernel
    chain), which alone leaves most CUs idle.  Steps on one lane stay in order (one stream), and a
    lane's static buffers are only rewritten by that lane's next step.  Nothing is shared between
    the lanes' graphs but the read-only weights (tests/test_lanes_gpu.py replays two lanes
    concurrently and checks every frame bitwise against sequential replays)."""

    def __init__(self, fn, example_inputs, lanes: int = 2, warmup: int = 2):
        if lanes < 1:
            raise ValueError("lanes >= 1")
        self.runners = [GraphRunner(lambda *x, _i=i: fn(_i, *x), example_inputs, warmup) for i in range(lanes)]
        self.streams = [torch.cuda.Stream() for _ in range(lanes)]
        self.k = 0

    @property
    def lanes(self):
        return len(self.runners)

    def next_lane(self) -> int:
        return self.k % len(self.runners)

    def replay(self):
        """One step on the next lane (inputs already in its static buffers); returns its outputs,
        valid once ``streams[lane]`` has run (``sync`` / ``join``)."""
        i = self.next_lane()
        self.k += 1
        with torch.cuda.stream(self.streams[i]):
            return self.runners[i].replay()

    def __call__(self, *inputs, out_fn=None):
        """One step on the next lane with ``inputs`` copied into its static buffers on the lane's
        stream (after the current stream's pending work, which produced them).  ``out_fn(outputs)``
        runs on the lane stream after the replay (e.g. copying the outputs out before the lane's
        next step rewrites them)."""
        i = self.next_lane()
        self.k += 1
        st = self.streams[i]
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            outs = self.runners[i](*inputs)
            if out_fn is not None:
                out_fn(outs)
            for t in inputs:                      # produced on the caller's stream, read on this one
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(st)
        return outs

    def join(self):
        """The current stream waits for every lane's steps so far."""
        cur = torch.cuda.current_stream()
        for st in self.streams:
            cur.wait_stream(st)
