"""Dry run of every engine's host plan on CPU: the ``torch.ops.s2v`` launch ops and the libs2v
entry points are replaced by no-ops that validate their arguments against the registered op
schemas (count, tensor-ness, int lists) / the C ABI's argument counts, so the shape / view / slice
bookkeeping of each forward (every NHWC assertion in ops.py) runs without a GPU.  Nothing is
computed — numerics are the gpu-marked tests' job; this catches plumbing errors before a GPU box is
spent on them."""
import ctypes

import pytest
import torch

import s2v_import  # noqa: F401
from helpers import GFPGAN_KW, synth_sd
from s2v_amd import _lib, ops, synth


class _NoLib:
    def __init__(self):
        self.calls = {}

    def __getattr__(self, name):
        if name not in _lib.EXPORTS:
            raise AttributeError(name)
        nargs = len(_lib._SIGS[name][1])

        def fn(*args):
            assert len(args) == nargs, f"{name}: {len(args)} args, ABI has {nargs}"
            self.calls[name] = self.calls.get(name, 0) + 1
            return 0
        return fn


class _NoOps:
    """Stand-in for torch.ops.s2v: each call is checked against the real op's schema."""

    def __init__(self, calls):
        from s2v_amd import torch_ops
        self.ns = torch_ops.load()
        self.calls = calls

    def __getattr__(self, name):
        schema = getattr(self.ns, name).default._schema
        args = schema.arguments

        def fn(*a, **kw):
            # positional arguments, then keywords; the rest must carry schema defaults
            names = [arg.name for arg in args]
            assert len(a) <= len(args) and all(k in names[len(a):] for k in kw), f"{name}: bad arguments {sorted(kw)}"
            for arg in args[len(a):]:
                assert arg.name in kw or arg.has_default_value(), f"{name}: missing {arg.name}"
            a = tuple(a) + tuple(kw.get(arg.name) if arg.name in kw else arg.default_value for arg in args[len(a):])
            for v, arg in zip(a, args):
                t = str(arg.type)
                if t == "Tensor":
                    assert isinstance(v, torch.Tensor), f"{name}.{arg.name}: tensor expected, got {type(v)}"
                elif t == "Optional[Tensor]":
                    assert v is None or isinstance(v, torch.Tensor), f"{name}.{arg.name}: tensor or None"
                elif t.startswith("List[int]"):
                    assert isinstance(v, (list, tuple)) and all(isinstance(i, int) for i in v), f"{name}.{arg.name}"
                elif t == "int":
                    assert isinstance(v, int), f"{name}.{arg.name}: int expected, got {type(v)}"
            self.calls[name] = self.calls.get(name, 0) + 1
            ret = str(schema.returns[0].type) if schema.returns else ""
            return [0] * 11 if ret.startswith("List") else 0 if ret == "int" else None
        return fn


@pytest.fixture
def dry(monkeypatch):
    lib = _NoLib()
    monkeypatch.setattr(ops, "S2V", _NoOps(lib.calls))
    monkeypatch.setattr(ops, "_require_cuda", lambda t, what: None)
    monkeypatch.setattr(ops._lib, "load", lambda: lib)
    monkeypatch.setattr(ops.Ctx, "stream", property(lambda self: ctypes.c_void_p(0)))
    return lib


def test_gfpgan_plan(dry):
    from s2v_amd.engine.gfpgan import GFPGANEngine
    eng = GFPGANEngine(synth_sd("gfpgan"), "cpu")
    x = torch.zeros(2, 3, 512, 512)
    out = torch.empty_like(x)
    for rn in (True, False):
        _, rgbs = eng.forward(ops.Ctx("cpu"), x, out, return_rgb=True, randomize_noise=rn)
    assert [r.shape[-1] for r in rgbs] == [8, 16, 32, 64, 128, 256, 512]
    assert dry.calls.get("modulated_conv2d_", 0) + dry.calls["conv2d_"] > 120 and dry.calls["eltwise_"] == 14   # the U-Net skip adds (SFT in the epilogues)


def test_gpen_plan(dry):
    from s2v_amd.engine.gpen import GPENEngine
    eng = GPENEngine(synth_sd("gpen"), "cpu")
    x = torch.zeros(2, 3, 512, 512)
    eng.forward(ops.Ctx("cpu"), x, torch.empty_like(x))
    assert dry.calls["fir2d_"] == 7 + 7 + 7 and dry.calls["eltwise_"] == 15  # the 15 noise-concat halves
    from s2v_amd.engine import gpen
    calls = dict(dry.calls)
    gpen.FOLD_NOISE, prev = True, gpen.FOLD_NOISE
    try:
        eng.forward(ops.Ctx("cpu"), x, torch.empty_like(x))
    finally:
        gpen.FOLD_NOISE = prev
    assert dry.calls["eltwise_"] - calls["eltwise_"] == 7     # folded: only the upsampling layers' halves


def test_lipsync_engines_plan(dry):
    from s2v_amd.engine.dnet import DNetEngine
    from s2v_amd.engine.enet import ENetEngine
    ctx = ops.Ctx("cpu")
    e = ENetEngine(synth_sd("enet"), "cpu")
    mel, face, gt = (torch.from_numpy(a) for a in synth.lipsync_inputs("dry", 2, 256))
    e.forward(ctx, mel, face, gt, torch.empty(2, 3, 384, 384), torch.empty(2, 3, 96, 96))
    d = DNetEngine(synth_sd("dnet"), "cpu")
    src, coeff = (torch.from_numpy(a) for a in synth.dnet_inputs("dry", 1, 256))
    d.forward(ctx, src, coeff)


def test_lnet_fused_ffc_plan(dry, monkeypatch):
    """LNet's 54 FFCs (3 levels x 9 blocks x 2) through the fused spectral / norm kernels (csrc/ffc.hip,
    S2V_LNET_FUSED=1) in f16x3: two spectral launches and one norm per FFC, no separate st1 / fu / st2 / FFT /
    InstanceNorm launches."""
    from s2v_amd.engine import lnet
    monkeypatch.setattr(lnet, "FUSED", True)
    monkeypatch.setattr(lnet, "FUSED_LEVELS", (12, 24, 48))
    eng = lnet.LNetEngine(synth_sd("lnet"), "cpu")
    mel, face, _ = (torch.from_numpy(a) for a in synth.lipsync_inputs("dry", 2, 96))
    x6 = ops.NHWC(face.permute(0, 2, 3, 1).contiguous())
    eng.forward(ops.Ctx("cpu"), mel, x6, ops.NHWC.empty(2, 96, 96, 3, "cpu"))
    assert dry.calls.get("ffc_spec_fwd_") == 54 and dry.calls.get("ffc_spec_inv_") == 54
    assert dry.calls.get("ffc_norm_") == 54 and "rfft2_" not in dry.calls and "instnorm_" not in dry.calls
    # PAIR (the default): conv_to_l and l2g of every FFC as one grouped launch
    assert dry.calls.get("group_end_", 0) >= 54 if lnet.PAIR else True     # (+ the grouped polyphase up convs)


def test_parsenet_plan(dry):
    from helpers import parsenet_sd
    from s2v_amd.engine.parsenet import ParseNetEngine
    from s2v_amd.models.parse_arch import ParseNetParams, face_parse_net
    desc = ParseNetParams(**face_parse_net(512)).describe()
    eng = ParseNetEngine(parsenet_sd(512), "cpu", desc)
    x = torch.zeros(2, 3, 512, 512)
    eng.forward(ops.Ctx("cpu"), x, torch.empty(2, 19, 512, 512), torch.empty(2, 3, 512, 512))
    # encoder conv + 4 down blocks (3 convs) + 10 body blocks (2) + 4 up blocks (3) + 2 heads
    assert dry.calls["conv2d_"] == 1 + 12 + 20 + 12 + 2 and dry.calls["eltwise_"] == 1


def test_perfdb_table_and_lookup(dry, monkeypatch):
    """The shipped perf-db (ops.PERFDB_PATH, tools/tune_perfdb.py) is well formed, and a conv whose
    conv_key() is in the table is launched with the table's forced (tile, split-K); an explicit
    force_tile, or a key not in the table, leaves the planner's choice (0, 0)."""
    import json
    import os
    with open(ops.PERFDB_PATH) as f:
        db = json.load(f)
    assert db["entries"] and set(db["workloads"]) >= {"lnet", "dnet", "lipsync", "enhance"}
    for k, v in db["entries"].items():
        assert k.startswith("x") and k.count("|") in (4, 5), k
        assert 1 <= v["tile"] <= 11 and v["splits"] in (1, 2, 3, 4, 6, 8, 12, 16), (k, v)
        assert v["us"] < 0.97 * v["planner_us"], (k, v)
    if os.environ.get("S2V_PERFDB", "1") != "0":
        assert len(ops.PERFDB) == len(db["entries"])
    seen = []
    real = ops.S2V

    class Rec:
        def __getattr__(self, name):
            fn = getattr(real, name)
            if name != "conv2d_":
                return fn

            def rec(*a):
                seen.append(tuple(a[31:33]))
                return fn(*a)
            return rec
    monkeypatch.setattr(ops, "S2V", Rec())
    # the table applies only on the device it was measured on (arch + CU count)
    assert db["arch"] == "gfx950" and db["cus"] == 256
    assert not ops.perfdb_applies("cpu")
    monkeypatch.setattr(ops, "perfdb_applies", lambda dev: True)
    prev = ops.set_precision("f16x3")
    try:
        ctx = ops.Ctx("cpu")
        x = ops.NHWC(torch.zeros(16, 14, 14, 64))
        cw = ops.ConvW(torch.zeros(96, 64, 3, 3), None, "cpu")
        y = ops.NHWC(torch.zeros(16, 12, 12, 96))
        key = ops.conv_key(x, cw, y.v, 1, False, ops.PREC_F16X3)
        monkeypatch.setattr(ops, "PERFDB", {key: (7, 12)})
        ops.conv2d(ctx, x, cw, y)
        ops.conv2d(ctx, x, cw, y, force_tile=2)
        monkeypatch.setattr(ops, "PERFDB", {key + "?": (7, 12)})
        ops.conv2d(ctx, x, cw, y)
    finally:
        ops.set_precision(prev)
    assert seen == [(7, 12), (2, 0), (0, 0)], seen
