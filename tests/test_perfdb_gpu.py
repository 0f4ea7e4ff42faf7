"""The conv perf-db (speech-to-video-mpp_amd/perfdb_mi355x.json, tools/tune_perfdb.py) forces tiles and
split-K factors the planner would not pick, at exactly the benchmarked shapes.  Each forced
configuration must compute the same convolution: the forward of each benchmarked workload with the
table must match the planner-only forward up to summation-order rounding, and the table must actually
be hit.  MI355X only."""
import sys

import pytest
import torch

import s2v_import  # noqa: F401
from s2v_amd import ops

pytestmark = pytest.mark.gpu


class _Counting(dict):
    hits = 0

    def get(self, k, default=None):
        if k in self:
            _Counting.hits += 1
        return super().get(k, default)


def _flat(out):
    if isinstance(out, torch.Tensor):
        return [out.detach().float().clone()]
    if isinstance(out, dict):
        out = list(out.values())
    if isinstance(out, (list, tuple)):
        return [t for o in out for t in _flat(o)]
    return []


@pytest.mark.parametrize("workload", ["lnet", "dnet", "enhance"])
def test_perfdb_matches_planner(workload, monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    args = bench.parse()
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[workload](args, dev, 0, 1)
    if workload == "enhance":     # the bench's GFPGAN draws fresh noise per forward; fixed noise here
        x = wl.inputs[0]

        def fn():
            return wl.gfpgan(x, return_rgb=False, randomize_noise=False)[0], wl.gpen(x)[0]
    else:
        fn = wl.forward
    table = _Counting(ops.PERFDB)
    assert table, "perf-db not loaded (S2V_PERFDB=0?)"
    with torch.no_grad():
        fn()                                           # range calibration
        monkeypatch.setattr(ops, "PERFDB", {})
        ref = _flat(fn())
        torch.cuda.synchronize()
        monkeypatch.setattr(ops, "PERFDB", table)
        _Counting.hits = 0
        got = _flat(fn())
        torch.cuda.synchronize()
    assert _Counting.hits > 0, f"{workload}: no launch matched a perf-db key"
    assert len(ref) == len(got) and ref
    for r, g in zip(ref, got):
        assert torch.isfinite(g).all()
        scale = max(1.0, float(r.abs().max()))
        err = float((r - g).abs().max())
        assert err <= 2e-3 * scale, f"{workload}: perf-db forward differs by {err:.3e} (scale {scale:.3g})"


@pytest.mark.parametrize("workload", ["lnet", "dnet", "enhance"])
def test_perfdb_each_forced_launch_matches_planner(workload, monkeypatch):
    """every conv launch of the workload whose key is in the table, run twice on the same
    inputs inside the launch hook (ops.TUNE) — once with the planner's configuration, once with the
    table's forced (tile, split-K) — must agree to fp32 summation-order rounding: max |diff| <= 2e-5 x
    max |planner output| per launch.  A forced configuration that dropped or duplicated a partial
    K-slice or a split-K edge would miss this by orders of magnitude (one 32-deep slice of a K >= 288
    conv is >= 1e-2 of the output)."""
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    args = bench.parse()
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[workload](args, dev, 0, 1)
    if workload == "enhance":
        x = wl.inputs[0]

        def fn():
            return wl.gfpgan(x, return_rgb=False, randomize_noise=False)[0], wl.gpen(x)[0]
    else:
        fn = wl.forward
    table = dict(ops.PERFDB)
    assert table and ops.perfdb_applies(dev)
    checked = []

    def hook(ctx, key, relaunch, plan_of, yv, resv):
        if key not in table or key in {k for k, _ in checked}:
            return
        tile, splits = table[key]
        torch.cuda.synchronize()
        saved = yv.clone()
        relaunch(0, 0)
        ref = yv.clone()
        yv.copy_(saved)
        relaunch(tile, splits)
        got = yv.clone()
        yv.copy_(saved)
        torch.cuda.synchronize()
        scale = float(ref.abs().max())
        err = float((ref - got).abs().max())
        checked.append((key, err / max(scale, 1e-30)))
    with torch.no_grad():
        fn()                                           # range calibration
        monkeypatch.setattr(ops, "TUNE", hook)
        fn()
        torch.cuda.synchronize()
    assert checked, f"{workload}: no launch matched a perf-db key"
    worst = max(checked, key=lambda c: c[1])
    assert worst[1] <= 2e-5, f"{workload}: forced launch {worst[0]} differs by {worst[1]:.3e} x max|out|"
