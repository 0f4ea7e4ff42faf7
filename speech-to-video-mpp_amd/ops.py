"""Tensor-level model-path ops: every kernel launch of the LNet / ENet / DNet / GFPGAN / GPEN
engines is a dispatch of a ``torch.ops.s2v`` custom op (csrc/torch_launch.cpp: TORCH_LIBRARY(s2v),
HIP kernel key), which validates the views and calls the C ABI of libs2v.so on the current HIP
stream.  torch.profiler therefore attributes the model path to ``s2v::*`` ops, like the reference's
aten ops under torch.no_grad() (inference.py:266), and a hipGraph capture records just the kernels.

PyTorch is used only as the dispatcher, device allocator and stream provider.  Inputs must be HIP
fp32 tensors; a CPU tensor raises (there is no CPU path in the product).

Layout: activations are NHWC tensors [N, H, W, Ctot]; an ``NHWC`` view selects a channel slice
[coff, coff + c) of one, which is how the reference's torch.cat / split / narrow disappear.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import os
import threading
import weakref

import torch

from . import _lib, torch_ops
from ._lib import (ACT_GELU_TANH, ACT_LRELU, ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH,  # noqa: F401
                   IN_DIRECT, IN_NEAREST_UP2, IN_TRANSPOSED, PAD_REFLECT, PAD_ZERO, PREC_BF16X3, PREC_F16X3, PREC_F32,
                   check)

F32 = 4

# Arithmetic of the implicit-GEMM convolutions (s2v_conv_params.prec):
#   "f16x3"  (default) split-fp32 on the f16 MFMA: 22 significant bits per operand, <= 3*2^-22
#            relative error per product for operands in the f16 normal range (weights are pre-scaled
#            into it by a power of two, undone exactly in the epilogue);
#   "bf16x3" split-fp32 on the bf16 MFMA: 16 significant bits per operand, <= 3*2^-16 per product,
#            any fp32 range;
#   "f32"    exact fp32 MFMA.
# All three run fp32 tensors with fp32 accumulation.  The S2V_PRECISION environment variable sets
# the process default; set_precision() changes it.
_PRECISIONS = {"f16x3": PREC_F16X3, "bf16x3": PREC_BF16X3, "f32": PREC_F32}
SPLIT_PRECISIONS = ("f16x3", "bf16x3")
PRECISION = os.environ.get("S2V_PRECISION", "f16x3")
if PRECISION not in _PRECISIONS:
    raise ValueError(f"S2V_PRECISION must be one of {sorted(_PRECISIONS)}, got {PRECISION!r}")


# f16x3 activation range guard.  The f16 halves of a split operand cover |v| < 65504, and a lo half
# becomes an f16 subnormal (absolute spacing 2^-24) once |v| < 2^-3.  Weights are pre-scaled by a
# power of two at packing (ConvW.split_scale); activations get a per-layer power-of-two pre-scale
# (s2v_conv_params.x_scale) chosen from the max |v| of the operand the kernel splits (the layer input,
# times max |in_scale| for a StyleGAN2 modulated input) on the engine's first forward: a layer whose
# max lies outside [X_LO, X_HI) is scaled so that it lands in [2^X_TARGET, 2^(X_TARGET + 1)), 64x below
# the f16 ceiling.  The first forward measures every layer into one device buffer and reads it with a
# single host sync (begin_calibration / end_forward); it is re-run with the scales when any layer needed
# one.  Every f16x3 launch also carries the lane's non-finite flag: an eager forward reads it when it
# returns (models._EngineMixin) and re-runs itself in bf16x3 (fp32's exponent range) when it is set; a
# graph-replayed pipeline batch copies it per batch and re-runs flagged batches the same way
# (pipeline.LipSyncPipeline.run) — an overflow is never silent and never left in the output.
# S2V_RANGE_GUARD=0 turns all of this off.
RANGE_GUARD = os.environ.get("S2V_RANGE_GUARD", "1") == "1"
X_LO, X_HI = 2.0 ** -3, 2.0 ** 14
X_TARGET = 9


def x_scale_for(amax: float) -> float:
    """Power-of-two activation pre-scale for a layer whose split operand has max |v| = ``amax``."""
    if not (amax > 0.0) or math.isinf(amax):
        return 1.0
    if X_LO <= amax < X_HI:
        return 1.0
    return float(2.0 ** (X_TARGET - math.floor(math.log2(amax))))


def set_precision(name: str) -> str:
    """Select the conv arithmetic ("f16x3", "bf16x3" or "f32") for launches issued from now on; returns the
    previous setting.  A captured HIP graph keeps the precision it was captured with."""
    global PRECISION
    if name not in _PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(_PRECISIONS)}, got {name!r}")
    prev, PRECISION = PRECISION, name
    return prev


@contextlib.contextmanager
def precision(name: str):
    """set_precision(name) for the launches issued inside the block."""
    prev = set_precision(name)
    try:
        yield
    finally:
        set_precision(prev)


def prec_code() -> int:
    return _PRECISIONS[PRECISION]

# Optional per-launch observer (bench.py's live roofline): called as hook(ctx, info, flops, launch)
# where info is the launch's ConvLaunch (kernel plan + shape) and launch() performs the conv; the
# hook may bracket it with events.
CONV_HOOK = None
# nearest-x2 polyphase convs (ConvW.make_up2_polyphase) whose input has at most this many pixels launch
# their four parity classes as one grouped kernel (conv_group)
UP2_GROUP_PIXELS = 16 * 48 * 48
# Optional launch timer (bench.py's roofline of the benchmarked, graph-replayed launches): called as
# STAMP(info, flops) for every conv launch (info: ConvLaunch); returns None or (stamps, stamp_ctr,
# [slot, stride, reps]) for the kernel's in-launch clock stamps (s2v_conv_params.stamps).
STAMP = None
_NOSTAMP = (None, None, [0, 1, 1])
# inside conv_group on this thread: launches are recorded (no per-launch stamps); thread-local like the
# C++ group recording it mirrors (torch_launch.cpp g_recording)
_TLS = threading.local()


def _grouping() -> bool:
    return getattr(_TLS, "grouping", False)
# Tuned (x3 tile, split-K) of split-precision conv launches whose planner choice (csrc/conv.hip
# make_plan_x3's time model) measured slower than another configuration: a table measured on MI355X by
# tools/tune_perfdb.py (every conv launch of the LNet / ENet / DNet forwards, each candidate tile and
# split factor graph-timed against the planner's own choice), keyed by conv_key().  Only entries that
# beat the planner by more than 3 % are kept; every other launch stays with the planner.
# S2V_PERFDB=0 ignores the table; S2V_PERFDB_PATH reads another one (A/B of tuned tables).
PERFDB_PATH = os.environ.get("S2V_PERFDB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                "perfdb_mi355x.json")
PERFDB = {}
PERFDB_DEVICE = None    # (arch, CU count) the table was measured on: applied only on a matching device
if os.environ.get("S2V_PERFDB", "1") != "0" and os.path.exists(PERFDB_PATH):
    import json as _json
    with open(PERFDB_PATH) as _f:
        _db = _json.load(_f)
    PERFDB = {k: (int(v["tile"]), int(v["splits"])) for k, v in _db["entries"].items()}
    PERFDB_DEVICE = (_db.get("arch"), _db.get("cus"))
_PERFDB_MATCH = {}


def perfdb_applies(device) -> bool:
    """The perf-db's forced tiles were timed on PERFDB_DEVICE (gfx950, 256 CUs): on another part the
    planner's own model decides (the key has no architecture or CU count in it)."""
    key = str(device)
    if key not in _PERFDB_MATCH:
        ok = False
        if PERFDB and torch.device(device).type == "cuda":
            pr = torch.cuda.get_device_properties(torch.device(device))
            ok = (pr.gcnArchName.split(":")[0], pr.multi_processor_count) == PERFDB_DEVICE
        _PERFDB_MATCH[key] = ok
    return _PERFDB_MATCH[key]
# tools/tune_perfdb.py: called as TUNE(ctx, key, relaunch, plan_of, yv, resv) for every launch conv_key()
# covers; relaunch(tile, splits) runs the conv with that forced configuration, plan_of(tile, splits) is its
# s2v_conv2d_plan (0, 0: the planner's own choice)
TUNE = None
LAST_GROUP = 0          # 1: the last conv_group launched as one grouped kernel, 0: one by one


class _Dispatch:
    """``torch.ops.s2v`` (libs2v_torch.so, loaded on first use).  tests/test_engine_dryrun.py swaps
    in a schema-checking stand-in to walk the engines' host plans on a machine without a GPU."""

    def __getattr__(self, name):
        return getattr(torch_ops.load(), name)


S2V = _Dispatch()


class ConvLaunch:
    """What one conv launch runs: ``plan`` = s2v_conv2d_plan's ten ints (kernel instance, split-K
    factor) plus the problem shape, for conv_symbol() / conv_splits() and the roofline hooks."""
    __slots__ = ("plan", "n", "h", "w", "cin", "oh", "ow", "cout", "kh", "kw", "in_scale", "nc_scale", "pix_add", "res",
                 "res_is_y")

    def __init__(self, plan, **kw):
        self.plan = list(plan)
        for k in self.__slots__[1:]:
            setattr(self, k, kw.get(k, 0))


_SIDE = threading.local()


@contextlib.contextmanager
def side_stream(stream, keep: list):
    """Run a forward's side branch on ``stream``: kernels launch there, but every tensor the branch
    allocates through ``empty`` / ``NHWC.empty`` comes from the *calling* stream and is appended to
    ``keep`` (alive until the caller drops the list, after the branch has been joined back).

    Why: the caching allocator puts an allocation made during a hipGraph capture into the graph's
    private pool only when its stream is recognised as capturing; a side stream forked into the
    capture is not reliably recognised on ROCm, so its tensors came from the global pool, went back
    there when the branch returned and were handed to the next forward or graph that allocated on
    that (pooled, recycled) stream — two graphs writing one buffer: the round-2 cross-engine
    corruption (tests/test_lanes_gpu.py).  Allocated on the capture stream they are graph-owned;
    kept alive to the join they are never reused while the branch still reads them."""
    prev = getattr(_SIDE, "v", None)
    # nested branches (a branch forking its own side streams) still allocate from the outermost calling
    # stream, the one the capture runs on
    _SIDE.v = (prev[0] if prev is not None else torch.cuda.current_stream(), keep)
    try:
        with torch.cuda.stream(stream):
            yield
    finally:
        _SIDE.v = prev


def empty(shape, device, dtype=torch.float32) -> torch.Tensor:
    """torch.empty for forward activations (side branches allocate from the calling stream)."""
    side = getattr(_SIDE, "v", None)
    if side is None:
        return torch.empty(shape, device=device, dtype=dtype)
    main, keep = side
    with torch.cuda.stream(main):
        t = torch.empty(shape, device=device, dtype=dtype)
    keep.append(t)
    return t


def _require_cuda(t: torch.Tensor, what: str):
    if not (t.is_cuda and t.dtype == torch.float32):
        raise _lib.S2VError(f"{what}: expected a float32 HIP device tensor, got {t.dtype} on {t.device} "
                            "(the s2v path has no CPU fallback)")


class NHWC:
    """Channel-slice view of a contiguous [N, H, W, Ctot] fp32 device tensor.  ``split``: 0, or the
    precision code (PREC_BF16X3 / PREC_F16X3) whose split-fp32 layout the tensor holds
    (s2v_split_act; only convolutions with x_split read it, and only in that same precision)."""
    __slots__ = ("t", "n", "h", "w", "cs", "coff", "c", "split")

    def __init__(self, t: torch.Tensor, coff: int = 0, c: int | None = None, split: int = 0):
        assert t.dim() == 4 and t.is_contiguous(), "NHWC view needs a contiguous 4-D tensor"
        _require_cuda(t, "NHWC")
        n_, h_, w_, c_ = t.shape
        canon = (h_ * w_ * c_, w_ * c_, c_, 1)
        if t.stride() != canon:       # contiguous with size-1 dims of arbitrary stride: canonical view
            t = t.as_strided(t.shape, canon)
        self.t = t
        self.n, self.h, self.w, self.cs = t.shape
        self.coff = coff
        self.c = self.cs - coff if c is None else c
        self.split = int(split)
        assert self.split in (0, PREC_BF16X3, PREC_F16X3), "split: 0 or a split precision code"
        assert 0 <= coff and coff + self.c <= self.cs
        assert not split or (coff % 32 == 0 and self.c % 32 == 0), "split views cover whole 32-channel blocks"

    @property
    def ptr(self) -> int:
        return self.t.data_ptr() + F32 * self.coff

    @property
    def v(self) -> torch.Tensor:
        """The view as a torch tensor [N, H, W, c] (a channel slice of ``t``)."""
        return self.t if (self.coff == 0 and self.c == self.cs) else self.t[..., self.coff: self.coff + self.c]

    def slice(self, coff: int, c: int) -> "NHWC":
        return NHWC(self.t, self.coff + coff, c, self.split)

    @staticmethod
    def empty(n, h, w, c, device) -> "NHWC":
        return NHWC(empty((n, h, w, c), device))


class Workspace:
    """Grow-only scratch buffer shared by the ops of one stream (split-K partials, norm stats).
    Grows only outside graph capture; a capture that needs more raises.  A replaced buffer is kept
    alive: HIP graphs captured earlier hold its address (an eager call of another shape — a ragged
    last batch — may grow the workspace after a capture; freeing the old one would leave those
    graphs writing into memory the allocator hands out again)."""

    def __init__(self, device):
        self.device = device
        self.buf = torch.empty(0, dtype=torch.uint8, device=device)
        self._retired = []

    def get(self, nbytes: int):
        if nbytes <= 0:
            return None, 0
        if self.buf.numel() < nbytes:
            if torch.device(self.device).type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise _lib.S2VError("workspace must be sized by an eager run before graph capture")
            if self.buf.numel() > 0:
                self._retired.append(self.buf)
            self.buf = torch.empty(int(nbytes * 1.25) + 256, dtype=torch.uint8, device=self.device)
        return self.buf.data_ptr(), self.buf.numel()

    def tensor(self):
        """The current buffer (uint8; None while empty) for the ops' ``Tensor? ws`` argument."""
        return self.buf if self.buf.numel() else None


def _with_ws(ctx, launch):
    """Run ``launch(ws)`` (an s2v op returning the workspace bytes it still needs, 0 = launched);
    grow the context's workspace once when it is short."""
    need = launch(ctx.ws.tensor())
    if need:
        ctx.ws.get(need)
        need = launch(ctx.ws.tensor())
        if need:
            raise _lib.S2VError(f"workspace of {ctx.ws.buf.numel()} bytes, the launch needs {need}")


class Ctx:
    """Execution context = one *lane*: device, workspace, and every piece of mutable device state a
    forward needs besides its activations — the side streams (each with its own Ctx, so split-K
    workspaces never alias across concurrent launches) and the noise draw counters.  Engines keep
    only read-only weights, so two Ctx objects can run forwards of the same engine concurrently
    (two captured graphs replayed on two streams): nothing either graph writes is shared."""

    ALL = weakref.WeakSet()          # every context (check_all_ranges)

    def __init__(self, device):
        self.device = torch.device(device)
        self.ws = Workspace(self.device)
        self.lib = _lib.load()
        self._streams = {}
        self._noise = {}
        self.keep = []          # the current forward's side-branch tensors (side_stream), dropped per forward
        self.parent = None      # side-branch contexts share their lane's range flag
        self.grid_cap = 0       # s2v_conv_params.grid_cap of this context's convs (x3_grid_cap)
        self.calib = None       # the lane's calibration forward in progress (begin_calibration)
        self.reruns = 0         # forwards re-run in bf16x3 after a range overflow (end_forward)
        self._flag = None
        Ctx.ALL.add(self)

    def range_flag(self):
        """The lane's non-finite flag (int32 [1], made eagerly on first use; None off-device)."""
        if self.parent is not None:
            return self.parent.range_flag()
        if self._flag is None:
            if self.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
                return None
            self._flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        return self._flag

    def check_range(self, what="s2v"):
        """Raise if a split-precision conv of this lane produced a non-finite value since the last
        check (activation range outside the calibrated pre-scale); resets the flag."""
        f = self._flag
        if f is None:
            return
        if int(f.item()):
            f.zero_()
            raise _lib.S2VError(f"{what}: a split-precision (f16x3) conv produced non-finite values: an activation "
                                "left the range calibrated on the first forward.  Re-calibrate (model.refresh()) "
                                "or run S2V_PRECISION=bf16x3 (fp32 exponent range)")

    def streams(self, key, n):
        """``n`` (stream, Ctx) pairs for the side branches of engine ``key`` (made once, CUDA
        devices only; None on other devices)."""
        if self.device.type != "cuda":
            return None
        if key not in self._streams:
            self._streams[key] = [(torch.cuda.Stream(self.device), Ctx(self.device)) for _ in range(n)]
            for _, c in self._streams[key]:
                c.parent = self
                c.keep = self.keep      # branch tensors live until the lane's next forward, like the lane's own
        assert len(self._streams[key]) >= n
        return self._streams[key][:n]

    def noise(self, key) -> "NoiseCounter":
        """The noise draw counter of engine ``key`` in this lane."""
        if key not in self._noise:
            self._noise[key] = NoiseCounter()
        return self._noise[key]

    @property
    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)


# ----------------------------------------------------------------------------- weights
def _pad2(t: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    out = torch.zeros((rows, cols), dtype=torch.float32)
    out[: t.shape[0], : t.shape[1]] = t
    return out


class ConvW:
    """Packed convolution weights [npad][kpad] with k = (ky*kw + kx)*cin + c, plus the folded
    per-output-channel epilogue scale/shift (bias, eval BatchNorm)."""

    def __init__(self, weight: torch.Tensor, bias=None, device="cuda", *, stride=1, padding=0, dilation=1,
                 transposed=False, output_padding=0, pad_mode=PAD_ZERO, in_mode=IN_DIRECT, bn=None, bn_eps=1e-5,
                 post_scale=None):
        w = weight.detach().to("cpu", torch.float32)
        if w.dim() == 2:
            w = w[:, :, None, None]
        elif w.dim() == 3:            # Conv1d [O, I, k] -> 1 x k
            w = w[:, :, None, :]
        if transposed:                # ConvTranspose2d [I, O, kh, kw] -> [O, I, kh, kw]
            w = w.transpose(0, 1)
            in_mode = IN_TRANSPOSED
        self.cout, self.cin, self.kh, self.kw = (int(s) for s in w.shape)
        self._w_oihw = w if in_mode in (IN_TRANSPOSED, IN_NEAREST_UP2) else None
        self.poly = None
        pair = lambda v: (v, v) if isinstance(v, int) else tuple(v)  # noqa: E731
        self.sh, self.sw = pair(stride)
        self.ph, self.pw = pair(padding)
        self.dh, self.dw = pair(dilation)
        if weight.dim() == 3:
            self.sh, self.ph, self.dh = 1, 0, 1
        self.oph, self.opw = pair(output_padding)
        self.pad_mode, self.in_mode = pad_mode, in_mode
        K = self.kh * self.kw * self.cin
        self.K = K
        self.kpad = (K + 31) // 32 * 32
        # rows padded so every N tile the planner may pick (BN <= 128, or 256 when cout > 128) reads
        # inside the packed buffer: the kernels load whole BN-row slabs of B without a row guard
        self.npad = (self.cout + 127) // 128 * 128 if self.cout <= 128 else (self.cout + 255) // 256 * 256
        wk = w.permute(0, 2, 3, 1).reshape(self.cout, K)
        self.wt = _pad2(wk, self.npad, self.kpad).to(device)
        scale = shift = None
        b = None if bias is None else bias.detach().to("cpu", torch.float32)
        if bn is not None:
            g, beta, mean, var = (t.detach().to("cpu", torch.float32) for t in bn)
            s = g / torch.sqrt(var + bn_eps)
            scale = s
            shift = beta - mean * s + (b * s if b is not None else 0.0)
        elif b is not None:
            shift = b
        if post_scale is not None:
            scale = (scale if scale is not None else torch.ones(self.cout)) * post_scale
            if shift is not None:
                shift = shift * post_scale
        self.scale = None if scale is None else scale.contiguous().to(device)
        self.shift = None if shift is None else shift.contiguous().to(device)

    _split = None

    def split_scale(self, prec: int) -> float:
        """Power-of-two pre-scale of the split weights (s2v_conv_params.wt_scale): f16 halves get
        max|W| into [2^13, 2^14) so every weight and its lo half stay in the f16 normal range; bf16
        has fp32's exponent range and needs none."""
        if prec != PREC_F16X3:
            return 1.0
        if getattr(self, "_f16_scale", None) is None:
            m = float(self.wt.abs().max())
            self._f16_scale = 1.0 if m == 0.0 else float(2.0 ** math.floor(math.log2(16384.0 / m)))
        return self._f16_scale

    def wt_x3(self, ctx: "Ctx", prec: int = PREC_BF16X3) -> torch.Tensor:
        """The packed weights in the split layout of ``prec`` (built once per precision, on first use)."""
        if self._split is None:
            self._split = {}
        if prec not in self._split:
            if self.wt.is_cuda and torch.cuda.is_current_stream_capturing():
                raise _lib.S2VError("split weights must be built by an eager run before graph capture")
            out = torch.empty(self.wt.shape, dtype=torch.float32, device=self.wt.device)
            S2V.split_weights_(self.wt, out, prec, self.split_scale(prec))
            self._split[prec] = out
        return self._split[prec]

    def make_polyphase(self, device):
        """Polyphase plan of a stride-2 ConvTranspose2d: output parity class (ry, rx) is a stride-1
        direct conv of the input with the taps ky = ry + p (mod 2), flipped, padded by T - 1 - c0
        (c0 = (ry + p - ky_min) / 2), written with output step 2 at offset (ry, rx).  Work drops
        from kh*kw taps per output pixel (3/4 of them zero) to the algorithmic count."""
        assert self.in_mode == IN_TRANSPOSED and (self.sh, self.sw) == (2, 2) and (self.dh, self.dw) == (1, 1)
        w = self._w_oihw
        plans = []
        for ry in range(2):
            ty = [k for k in range(self.kh) if (ry + self.ph - k) % 2 == 0]
            for rx in range(2):
                tx = [k for k in range(self.kw) if (rx + self.pw - k) % 2 == 0]
                if not ty or not tx:
                    raise NotImplementedError("polyphase class without taps")
                c0y, c0x = (ry + self.ph - ty[0]) // 2, (rx + self.pw - tx[0]) // 2
                sub = w[:, :, ty[::-1]][:, :, :, tx[::-1]]
                cw = ConvW(sub, None, device, padding=(len(ty) - 1 - c0y, len(tx) - 1 - c0x))
                cw.scale, cw.shift = self.scale, self.shift
                plans.append(((ry, rx), cw, (ry, rx)))
        self.poly = plans
        return self

    # nearest-x2 3x3 fold: source offset a of output parity r collects the conv taps k with F[r][a][k] = 1
    _UP2_FOLD = (((1, 0, 0), (0, 1, 1)), ((1, 1, 0), (0, 0, 1)))

    def make_up2_polyphase(self, device):
        """Polyphase plan of a 3x3 stride-1 zero-padded conv over a nearest-x2 upsampled input
        (IN_NEAREST_UP2: UpBlock2d, models/base_blocks.py:104-118, LNet / DNet decoders).  Output parity
        class (ry, rx) only reads the 2x2 source pixels its taps land on, so it is a 2x2 conv of the
        un-upsampled input with the taps that hit one source pixel summed (parity 0: source offsets
        {-1, 0} with weights {w0, w1 + w2}, padding 1; parity 1: {0, +1} with {w0 + w1, w2}, padding 0),
        written with output step 2 at offset (ry, rx) like a transposed conv's classes (``poly``).
        4/9 of the direct conv's multiply-adds, and each class takes the buffer-load A path instead of
        the per-row upsample gather; the 2x2 tap sums are formed in fp64 and rounded once."""
        assert self.in_mode == IN_NEAREST_UP2 and (self.kh, self.kw) == (3, 3) and (self.ph, self.pw) == (1, 1)
        assert (self.sh, self.sw, self.dh, self.dw) == (1, 1, 1, 1) and self.pad_mode == PAD_ZERO
        f = torch.tensor(self._UP2_FOLD, dtype=torch.float64)
        w = self._w_oihw.double()
        plans = []
        for ry in range(2):
            for rx in range(2):
                sub = torch.einsum("ap,bq,oipq->oiab", f[ry], f[rx], w).float()
                cw = ConvW(sub, None, device, padding=(1 - ry, 1 - rx))
                cw.scale, cw.shift = self.scale, self.shift
                plans.append(((ry, rx), cw, (ry, rx)))
        self.poly = plans
        return self

    def make_rowpack(self, device):
        """Row-tap packed form of a kh x kw stride-1 zero-padded conv over c <= 8 channels: the input is
        packed by ``row_pack`` into kw * c channels (padded to a multiple of 32) and the conv runs as a
        kh x 1 conv whose weight channel dx * c + ci holds tap (ky, dx) of input channel ci — the same
        products and sums (in a different order), on the buffer-load tiles instead of the per-element
        gather that small channel counts otherwise take."""
        assert self.in_mode == IN_DIRECT and (self.sh, self.sw, self.dh, self.dw) == (1, 1, 1, 1)
        assert self.pad_mode == PAD_ZERO and self.cin * self.kw <= 64 and 2 * self.pw + 1 == self.kw
        w = self.wt[: self.cout, : self.K].cpu().reshape(self.cout, self.kh, self.kw, self.cin)   # [o, ky, kx, ci]
        cp = (self.kw * self.cin + 31) // 32 * 32
        wp = torch.zeros(self.cout, cp, self.kh, 1)
        wp[:, : self.kw * self.cin, :, 0] = w.permute(0, 2, 3, 1).reshape(self.cout, self.kw * self.cin, self.kh)
        cw = ConvW(wp, None, device, padding=(self.ph, 0))
        cw.scale, cw.shift = self.scale, self.shift
        self.rowpack = cw
        return self

    rowpack = None

    def out_hw(self, h, w):
        if self.in_mode == IN_TRANSPOSED:
            return ((h - 1) * self.sh - 2 * self.ph + self.dh * (self.kh - 1) + self.oph + 1,
                    (w - 1) * self.sw - 2 * self.pw + self.dw * (self.kw - 1) + self.opw + 1)
        if self.in_mode == IN_NEAREST_UP2:
            h, w = 2 * h, 2 * w
        return ((h + 2 * self.ph - self.dh * (self.kh - 1) - 1) // self.sh + 1,
                (w + 2 * self.pw - self.dw * (self.kw - 1) - 1) // self.sw + 1)


def _ptr(t):
    return None if t is None else t.data_ptr()


def conv2d(ctx: Ctx, x: NHWC, cw: ConvW, y: NHWC, *, act=ACT_NONE, alpha=0.0, res: NHWC | None = None,
           res_after=False, res_offset=(0, 0), nc_scale=None, in_scale=None, pre_act=ACT_NONE, pre_alpha=0.0,
           pix_add=None, pix_w=0.0, scale=None, shift=None, force_tile=0, force_splits=0, pool=False, post=None,
           dup=None):
    """Fused conv (s2v_conv_params, dispatched as ``s2v::conv2d_``).  nc_scale / in_scale: [N, C]
    device tensors.  A transposed ConvW with a polyphase plan (``cw.poly``) runs as one stride-1 conv
    per output parity class, each writing every second pixel of y.  ``pool``: y is the 2x2 average
    pool of the activated conv output (half the conv's size).
    ``post`` = (mul, add, c0): SFT on output channels >= c0 after the activation, y = v * mul + add with
    mul / add NHWC views of y's pixels over cout - c0 channels (gfpganv1_clean_arch.py:98-106).
    ``dup`` = (src, bias, a, off): a second output y.t[..., off + n] = act(a * src[..., n] + bias[n]) in
    the same epilogue, src an NHWC view of y's pixels over cout channels (GPEN's noise-injection concat
    half, gpen_model.py:292-302)."""
    assert (post is None and dup is None) or (cw.rowpack is None and getattr(cw, "poly", None) is None), \
        "conv: post / dup epilogues on plain (not row-packed, not polyphase) convs only"
    if cw.rowpack is not None:
        # small-channel wide-kernel conv: row-tap packed input, kh x 1 conv over the packed channels
        assert x.c == cw.cin, f"conv: input has {x.c} channels, weights expect {cw.cin}"
        assert in_scale is None, "row-packed conv: no input scale"
        xp = NHWC.empty(x.n, x.h, x.w, cw.rowpack.cin, x.t.device)
        row_pack(ctx, x, xp, cw.kw, cw.pw)
        return conv2d(ctx, xp, cw.rowpack, y, act=act, alpha=alpha, res=res, res_after=res_after, res_offset=res_offset,
                      nc_scale=nc_scale, in_scale=None, pre_act=pre_act, pre_alpha=pre_alpha, pix_add=pix_add,
                      pix_w=pix_w, scale=scale, shift=shift, force_tile=force_tile, force_splits=force_splits, pool=pool)
    if getattr(cw, "poly", None) is not None:
        assert pix_add is None, "polyphase transposed conv: no pix_add epilogue"
        assert res is None or (res.t.data_ptr() == y.t.data_ptr() and res.coff == y.coff and not res_after), \
            "polyphase transposed conv: only an in-place residual (res is the output view)"
        oh, ow = cw.out_hw(x.h, x.w)
        assert (y.n, y.h, y.w, y.c) == (x.n, oh, ow, cw.cout), "conv_transpose: output view mismatch"
        # the four classes of a small nearest-x2 conv (LNet's decoder up convs) as one grouped launch
        grouped = cw.in_mode == IN_NEAREST_UP2 and x.n * x.h * x.w <= UP2_GROUP_PIXELS and not force_tile
        with conv_group(ctx, enabled=grouped):
            for (ry, rx), sub, _ in cw.poly:
                if (oh - ry + 1) // 2 <= 0 or (ow - rx + 1) // 2 <= 0:
                    continue
                yc = y.t[:, ry::2, rx::2, y.coff: y.coff + y.c]          # one output parity class
                _conv(ctx, x, sub, yc, 2, act, alpha, yc if res is not None else None, False, (0, 0), nc_scale,
                      in_scale, pre_act, pre_alpha, None, 0.0, scale, shift, force_tile, force_splits)
        return y
    oh, ow = cw.out_hw(x.h, x.w)
    assert x.c == cw.cin, f"conv: input has {x.c} channels, weights expect {cw.cin}"
    f = 2 if pool else 1
    assert (y.n, y.h * f, y.w * f, y.c) == (x.n, oh, ow, cw.cout), \
        f"conv: output view {(y.n, y.h, y.w, y.c)} != {(x.n, oh // f, ow // f, cw.cout)}"
    extra = {}
    if post is not None:
        pm, pa, c0 = post
        assert (pm.n, pm.h, pm.w, pm.c) == (y.n, y.h, y.w, cw.cout - c0) and (pa.n, pa.h, pa.w, pa.c) == (pm.n, pm.h,
                                                                                                         pm.w, pm.c)
        extra.update(post_mul=pm.v, post_add=pa.v, post_c0=int(c0))
    if dup is not None:
        ds, db, da, off = dup
        assert (ds.n, ds.h, ds.w, ds.c) == (y.n, y.h, y.w, cw.cout)
        assert y.coff == 0 and off >= cw.cout and off + cw.cout <= y.cs, "dup: second output inside y's pixel pitch"
        extra.update(dup_src=ds.v, dup_bias=db, dup_a=float(da), dup_off=int(off))
    _conv(ctx, x, cw, y.v, 1, act, alpha, None if res is None else res.v, res_after, res_offset, nc_scale, in_scale,
          pre_act, pre_alpha, pix_add, pix_w, scale, shift, force_tile, force_splits, pool=pool, extra=extra)
    return y


def _conv_flops(x, cw, yv, pool):
    """Algorithmic FLOPs (2 MAC) of one launch; a transposed conv counts only its real taps."""
    oh, ow = (yv.shape[1], yv.shape[2])
    if pool:
        oh, ow = 2 * oh, 2 * ow
    pix = x.n * x.h * x.w if cw.in_mode == IN_TRANSPOSED else x.n * oh * ow
    return 2.0 * pix * cw.kh * cw.kw * cw.cin * cw.cout


def conv_key(x, cw, yv, out_step, pool, prec) -> str:
    """Signature of a conv launch for PERFDB: input view geometry, filter geometry and modes, output
    view geometry, output step / pool, precision code (what the planner's choice depends on)."""
    return (f"x{x.n}x{x.h}x{x.w}x{x.c}c{x.cs}|k{cw.kh}x{cw.kw}s{cw.sh}x{cw.sw}p{cw.ph}x{cw.pw}d{cw.dh}x{cw.dw}"
            f"m{cw.in_mode}{cw.pad_mode}|y{yv.shape[1]}x{yv.shape[2]}x{cw.cout}c{yv.stride(2)}|o{out_step}{int(pool)}"
            f"|p{prec}")


def _conv(ctx, x, cw, yv, out_step, act, alpha, resv, res_after, res_offset, nc_scale, in_scale, pre_act, pre_alpha,
          pix_add, pix_w, scale, shift, force_tile, force_splits, pool=False, extra=None):
    """One ``s2v::conv2d_`` launch: x an NHWC view, yv / resv torch views (out_step 2: a strided
    parity-class view of a wider tensor)."""
    prec = prec_code()
    x_split = int(getattr(x, "split", 0))
    if x_split and x_split != prec:
        raise _lib.S2VError(f"conv: the input holds the split layout of precision code {x_split}, but the conv runs "
                            f"in {PRECISION!r} (code {prec}); split it again with split_act after set_precision")
    wsplit = cw.wt_x3(ctx, prec) if prec != PREC_F32 else None
    wscale = cw.split_scale(prec)
    xscale, flag = _range(ctx, cw, x, prec, in_scale)
    cap = int(getattr(ctx, "grid_cap", 0))
    sc = cw.scale if scale is None else scale
    sh = cw.shift if shift is None else shift
    key = None
    if (PERFDB or TUNE is not None) and prec != PREC_F32 and not (force_tile or force_splits or x_split or cap or
                                                                   _grouping()):
        key = conv_key(x, cw, yv, out_step, pool, prec)
        if TUNE is None and perfdb_applies(x.t.device):
            force_tile, force_splits = PERFDB.get(key, (0, 0))

    def launch(ws, dry=False, st=_NOSTAMP, ft=None, fs=None):
        return S2V.conv2d_(x.v, yv, cw.wt, wsplit, wscale, cw.cout, [cw.kh, cw.kw], [cw.sh, cw.sw], [cw.ph, cw.pw],
                           [cw.dh, cw.dw], cw.in_mode, cw.pad_mode, prec, sc, sh, in_scale, nc_scale, pre_act, pre_alpha,
                           pix_add, pix_w, resv, list(res_offset), res_after, act, alpha, out_step, pool, x_split != 0,
                           ws, cap, force_tile if ft is None else ft, force_splits if fs is None else fs, st[0], st[1],
                           st[2], xscale, flag, dry, **(extra or {}))
    if TUNE is not None and key is not None:
        TUNE(ctx, key, lambda ft, fs: _with_ws(ctx, lambda ws: launch(ws, False, _NOSTAMP, ft, fs)[0]),
             lambda ft, fs: launch(ctx.ws.tensor(), True, _NOSTAMP, ft, fs)[1:], yv, resv)
    _run_conv(ctx, launch, x, cw, yv, pool, in_scale, nc_scale, pix_add, resv)


@contextlib.contextmanager
def conv_group(ctx: Ctx, enabled: bool = True):
    """Launch the convs issued on ``ctx`` inside the block as ONE grouped kernel (s2v_conv2d_group:
    independent convs that read the same input, each with its own split-K factor, plus one grouped
    split-K fold) at the end of the block.  The members must not depend on each other.  Off when
    ``enabled`` is false or a CONV_HOOK observes launches (the roofline pre-pass times convs one by
    one): then the convs launch as they are issued."""
    if not enabled or CONV_HOOK is not None:
        yield
        return
    S2V.group_begin_()
    _TLS.grouping = True
    try:
        yield
    except BaseException:
        S2V.group_abort_()
        raise
    finally:
        _TLS.grouping = False
    global LAST_GROUP
    res = []

    def end(ws):
        r = S2V.group_end_(ws, False)
        res[:] = r
        return r[0]
    try:
        _with_ws(ctx, end)
    except BaseException:
        S2V.group_abort_()
        raise
    LAST_GROUP = res[1] if len(res) > 1 else 0


def check_all_ranges(what="s2v"):
    """Ctx.check_range over every live context (raises on the first flagged lane)."""
    for c in list(Ctx.ALL):
        c.check_range(what)


def guard_active() -> bool:
    """The f16x3 range guard applies to launches issued now."""
    return RANGE_GUARD and PRECISION == "f16x3"


class _Calibration:
    """Layers measured during one calibration forward: amax slots in one device buffer."""
    SLOTS = 4096

    def __init__(self, device):
        self.device = device
        self.bufs = [torch.zeros(self.SLOTS, device=device)]
        self.n = 0
        self.items = []          # (cw, prec, x slot, in_scale slot or -1)

    def slot(self):
        if self.n == len(self.bufs) * self.SLOTS:
            self.bufs.append(torch.zeros(self.SLOTS, device=self.device))
        i = self.n
        self.n += 1
        return i, self.bufs[i // self.SLOTS][i % self.SLOTS: i % self.SLOTS + 1]


def _root(ctx):
    while getattr(ctx, "parent", None) is not None:
        ctx = ctx.parent
    return ctx


def _amax_into(t: torch.Tensor, out: torch.Tensor):
    """max |t| of an NHWC view (4-D) or an [N, C] row view (2-D) into out (float32 [1])."""
    if t.dim() == 2:
        n, c = t.shape
        t = t.as_strided((1, 1, n, c), (n * t.stride(0), n * t.stride(0), t.stride(0), 1))
    S2V.amax_(t, out)


# calibration passes of an engine's first eager forward beyond the first (models._EngineMixin._guarded):
# each pass measures the layers an upstream overflow left unmeasured; past the limit the forward runs in
# bf16x3
CALIB_PASSES = 4


def begin_calibration(ctx):
    """Start a calibration forward on ``ctx``'s lane: uncalibrated f16x3 layers launch unscaled and
    record their operand's max |v| (no host sync) until end_forward."""
    _root(ctx).calib = _Calibration(ctx.device)


def end_forward(ctx, calibrating: bool) -> str:
    """After an eager forward on ``ctx``'s lane (one host sync): apply the measured scales of a
    calibration forward and read + clear the lane's non-finite flag.  Returns "recalibrate" when a layer
    measured a non-finite operand (an upstream layer overflowed before its own pre-scale existed: the
    layer stays uncalibrated and the next forward must be a calibration forward again, which measures it
    behind the now-scaled upstream layers), "scaled" when the forward must run again because a layer now
    carries a pre-scale, "overflow" when a launch produced a non-finite value (run the forward again in
    bf16x3), "" otherwise."""
    root = _root(ctx)
    cal = getattr(root, "calib", None) if calibrating else None
    root.calib = None
    flag = root._flag
    vals = [b.cpu() for b in cal.bufs] if cal is not None else []
    bad = bool(int(flag.item())) if flag is not None else False
    if flag is not None and bad:
        flag.zero_()
    scaled = False
    if cal is not None:
        per = {}
        for cw, prec, xs, ss in cal.items:
            m = float(vals[xs // _Calibration.SLOTS][xs % _Calibration.SLOTS])
            if ss >= 0:
                m *= float(vals[ss // _Calibration.SLOTS][ss % _Calibration.SLOTS])
            key = (id(cw), prec)
            per[key] = (cw, prec, max(per[key][2], m) if key in per else m)
        recal = False
        for cw, prec, m in per.values():
            if not math.isfinite(m):
                recal = True                  # left uncalibrated: measured again by the next calibration pass
                continue
            sc = x_scale_for(m)
            cw.__dict__.setdefault("_xscale", {})[prec] = sc
            cw.x_amax = m
            scaled = scaled or sc != 1.0
        if recal:
            return "recalibrate"
    if scaled:
        return "scaled"
    return "overflow" if bad else ""


def _range(ctx, cw, x, prec, in_scale=None):
    """(x_scale, flag) of an f16x3 launch: the layer's calibrated activation pre-scale and the lane's
    non-finite flag.  An uncalibrated layer is measured: into the lane's calibration buffer during a
    calibration forward (launched unscaled), else on the spot with one host sync."""
    if prec != PREC_F16X3 or not RANGE_GUARD or int(getattr(x, "split", 0)):
        return 1.0, None
    scales = cw.__dict__.setdefault("_xscale", {})
    s = scales.get(prec)
    if s is None:
        if x.t.is_cuda and torch.cuda.is_current_stream_capturing():
            raise _lib.S2VError("activation ranges must be calibrated by an eager run before graph capture")
        cal = getattr(_root(ctx), "calib", None)
        if cal is not None:
            xs, out = cal.slot()
            _amax_into(x.v, out)
            ss = -1
            if in_scale is not None:
                ss, out2 = cal.slot()
                _amax_into(in_scale, out2)
            cal.items.append((cw, prec, xs, ss))
            return 1.0, ctx.range_flag()
        m = torch.zeros(2, device=x.t.device)
        _amax_into(x.v, m[0:1])
        if in_scale is not None:
            _amax_into(in_scale, m[1:2])
        mv = m.cpu()
        amax = float(mv[0]) * (float(mv[1]) if in_scale is not None else 1.0)
        s = x_scale_for(amax)
        scales[prec] = s
        cw.x_amax = amax
    return s, ctx.range_flag()


def _run_conv(ctx, launch, x, cw, yv, pool, in_scale=None, nc_scale=None, pix_add=None, resv=None):
    st = _NOSTAMP

    def go():
        _with_ws(ctx, lambda ws: launch(ws, False, st)[0])
    if CONV_HOOK is None and STAMP is None:
        go()
        return
    plan = launch(ctx.ws.tensor(), True)[1:]
    oh, ow = yv.shape[1] * (2 if pool else 1), yv.shape[2] * (2 if pool else 1)
    info = ConvLaunch(plan, n=x.n, h=x.h, w=x.w, cin=x.c, oh=oh, ow=ow, cout=cw.cout, kh=cw.kh, kw=cw.kw,
                      in_scale=in_scale is not None, nc_scale=nc_scale is not None, pix_add=pix_add is not None,
                      res=resv is not None, res_is_y=resv is not None and resv.data_ptr() == yv.data_ptr())
    flops = _conv_flops(x, cw, yv, pool)
    if STAMP is not None and not _grouping():
        st = STAMP(info, flops) or _NOSTAMP
    if CONV_HOOK is None:
        go()
    else:
        CONV_HOOK(ctx, info, flops, go)


def modulate_weights(ctx: Ctx, cw: ConvW, s: torch.Tensor, d: torch.Tensor | None, batch: int):
    """The per-sample weights W * s[b, c] (* d[b, o]) of ``cw`` alone (``s2v::modulate_weights_``), in the layout a
    split-precision modulated conv reads (pre-scale 2^11 when demodulated in f16x3), or fp32 in f32 mode: the
    (wbuf, premod) pair modulated_conv2d(premod=) takes, so the modulation can run ahead of the conv (e.g. on a
    side stream as soon as the style code exists)."""
    prec = prec_code()
    wbuf = empty((batch, cw.npad, cw.kpad), cw.wt.device)      # (calling-stream memory on a side branch)
    wscale = 2048.0 if (prec == PREC_F16X3 and d is not None) else 1.0
    S2V.modulate_weights_(cw.wt, s, d, wbuf, cw.cout, cw.cin, cw.kh * cw.kw, prec, wscale)
    return wbuf, (wscale if prec != PREC_F32 else -1.0)


def modulated_conv2d(ctx: Ctx, x: NHWC, cw: ConvW, y: NHWC, s: torch.Tensor, d: torch.Tensor | None = None, *,
                     act=ACT_NONE, alpha=0.0, res: NHWC | None = None, res_after=False, pix_add=None, pix_w=0.0,
                     shift=None, force_splits=0, d2s=False, premod=None):
    """StyleGAN2 modulated conv with per-sample weights W * s[b, c] (* d[b, o]) written by the
    ``s2v::modulated_conv2d_`` op in the form its planned kernel reads (split layout with a 2^11 f16
    pre-scale when demodulated, or fp32), then one batched conv (no prologue / epilogue scaling in
    the GEMM).  s: [B, cin] (row stride s.stride(0)); d: [B, cout] demodulation or None.
    ``d2s``: cw holds the 4 parity classes of a x2-upsampled conv (cout = 4 classes x c, class-major)
    and y is the full [B, 2H, 2W, c] output (s2v_conv_params.d2s_cout); pix_add is then [B, 2H, 2W].
    ``premod``: a (wbuf, premod) pair from modulate_weights for the same (cw, s, d): the conv reads those weights
    instead of modulating them again (the op refuses a layout its plan does not read)."""
    oh, ow = cw.out_hw(x.h, x.w)
    assert cw.in_mode != IN_TRANSPOSED and cw.poly is None and (cw.sh, cw.sw, cw.dh, cw.dw) == (1, 1, 1, 1), \
        "modulated_conv2d: direct stride-1 convs only"
    if d2s:
        assert x.c == cw.cin and cw.cout % 4 == 0 and res is None and (y.n, y.h, y.w, y.c) == (x.n, 2 * oh, 2 * ow,
                                                                                             cw.cout // 4)
    else:
        assert x.c == cw.cin and (y.n, y.h, y.w, y.c) == (x.n, oh, ow, cw.cout)
    if premod is not None:
        wbuf, pm = premod
        assert tuple(wbuf.shape) == (x.n, cw.npad, cw.kpad), "modulated_conv2d: premod weights of another shape"
    else:
        wbuf, pm = torch.empty((x.n, cw.npad, cw.kpad), device=cw.wt.device), 0.0
    yv, resv = y.v, None if res is None else res.v
    prec = prec_code()
    x_split = int(getattr(x, "split", 0))
    if x_split and x_split != prec:
        raise _lib.S2VError(f"modulated conv: the input holds the split layout of precision code {x_split}, but the "
                            f"conv runs in {PRECISION!r} (code {prec})")
    sh = cw.shift if shift is None else shift            # the layer bias (epilogue shift) unless overridden
    xscale, flag = _range(ctx, cw, x, prec)
    key, force_tile = None, 0
    if (PERFDB or TUNE is not None) and prec != PREC_F32 and not (force_splits or x_split):
        key = conv_key(x, cw, yv, 1, False, prec) + f"|mod{int(d is not None)}{int(d2s)}"
        if TUNE is None and perfdb_applies(x.t.device):
            force_tile, force_splits = PERFDB.get(key, (0, 0))

    def launch(ws, dry=False, st=_NOSTAMP, ft=None, fs=None):
        return S2V.modulated_conv2d_(x.v, yv, cw.wt, s, d, wbuf, cw.cout, [cw.kh, cw.kw], [cw.ph, cw.pw], cw.in_mode,
                                     prec,
                                     x_split != 0, cw.scale, sh, pix_add, pix_w, resv, res_after, act, alpha, ws,
                                     force_splits if fs is None else fs, st[0], st[1], st[2], xscale, flag, dry, int(d2s),
                                     force_tile if ft is None else ft, pm)
    if TUNE is not None and key is not None:
        TUNE(ctx, key, lambda ft, fs: _with_ws(ctx, lambda ws: launch(ws, False, _NOSTAMP, ft, fs)[0]),
             lambda ft, fs: launch(ctx.ws.tensor(), True, _NOSTAMP, ft, fs)[1:], yv, resv)
    # roofline accounting on the conv's own grid (one parity class of y x all 4 x c columns = the
    # upsampled conv's FLOPs)
    _run_conv(ctx, launch, x, cw, yv[:, ::2, ::2, :] if d2s else yv, False, pix_add=pix_add, resv=resv)
    return y


def gemm_kn(ctx: Ctx, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, *, batch: int, a_bs: int, b_bs: int,
            out_bs: int, res: torch.Tensor | None = None, res_bs: int = 0, act=ACT_NONE, alpha=0.0,
            force_tile=0, force_splits=0):
    """Batched out[z] = a[z] @ b[z] (+res[z]) with a [M, K] row-major (K contiguous, lda = K),
    b [K, N] row-major (ldb = N), out [M, N] (ldc = N) (``s2v::gemm_kn_``)."""
    prec = prec_code()
    _with_ws(ctx, lambda ws: S2V.gemm_kn_(a, b, out, batch, a_bs, b_bs, out_bs, res, res_bs, act, alpha, prec, ws,
                                          force_tile, force_splits, False)[0])
    return out


def _plan(ctx: Ctx, p):
    out = (ctypes.c_int * 11)()
    check(ctx.lib.s2v_conv2d_plan(ctypes.byref(p), out), "s2v_conv2d_plan")
    return list(out)


def plan_symbol(plan) -> str:
    """Kernel symbol (as rocprofv3 reports it, demangled) of a launch plan (s2v_conv2d_plan's eleven ints)."""
    bm, bn, wm, avec, bkn, splits, x3, nw, ks, pf = plan[:10]
    persist = plan[10] if len(plan) > 10 else 0
    if avec == 5:
        return f"void s2v::conv_glds_x3<{bm}, {bn}, {wm}, {ks}, {x3 - 1}>(s2v::ConvArgs)"
    if avec in (6, 7):
        return f"void s2v::conv_x3_nar<{x3 - 1}, {avec - 6}>(s2v::ConvArgs)"
    if avec == 8:
        return f"void s2v::conv_x3_halo<{x3 - 1}, {bm // 64}, {bn // 64}>(s2v::ConvArgs)"
    if bm == 0:
        if wm < 0:
            if bkn >= 2000:
                return f"void s2v::conv_smallk4<{-wm}, {bkn - 2000}>(s2v::ConvArgs, int, int, int, int)"
            return f"void s2v::conv_smallk<{-wm}, {avec}>(s2v::ConvArgs, int, int, int, int)"
        if bkn >= 4000:
            return f"void s2v::conv_k4_mfma<{bkn - 4000}, false>(s2v::ConvArgs, int)"
        if bkn >= 3000:
            return f"void s2v::conv_head_x3<{x3 - 1}, {bn}, {bkn - 3000}, {wm}>(s2v::ConvArgs, int, int)"
        if bkn >= 1000:
            return f"void s2v::conv_halo_small<{bn}, {bkn - 1000}>(s2v::ConvArgs, int, int)"
        if wm:
            return f"void s2v::conv_small_cpar<{bn}, {wm}, {'true' if avec else 'false'}>(s2v::ConvArgs, int)"
        return f"void s2v::conv_direct_small<{bn}>(s2v::ConvArgs, int)"
    if x3:
        name = "conv_igemm_x3_persist" if persist else "conv_igemm_x3"
        return f"void s2v::{name}<{bm}, {bn}, {wm}, {nw}, {ks}, {pf}, {avec}, {bkn}, {x3 - 1}>(s2v::ConvArgs)"
    return f"void s2v::conv_igemm<{bm}, {bn}, {wm}, {avec}, {bkn}>(s2v::ConvArgs)"


def conv_symbol(ctx: Ctx, p) -> str:
    """Kernel symbol the launch ``p`` runs (a ConvLaunch from CONV_HOOK, or raw s2v_conv_params)."""
    return plan_symbol(p.plan if isinstance(p, ConvLaunch) else _plan(ctx, p))


def split_act(ctx: Ctx, x: NHWC, out: NHWC | None = None) -> NHWC:
    """fp32 activations -> the split layout of the current precision (``s2v::split_act_``), the
    input form of the LDS-DMA convolutions.  ``out``: a whole contiguous tensor of x's shape."""
    prec = prec_code()
    assert prec != PREC_F32, "split_act needs a split precision (f16x3 / bf16x3)"
    if out is None:
        out = NHWC.empty(x.n, x.h, x.w, x.c, x.t.device)
    assert (out.n, out.h, out.w, out.c) == (x.n, x.h, x.w, x.c) and out.coff == 0
    S2V.split_act_(x.v, out.v, prec)
    out.split = prec
    return out


(TUNE_HALO_MIN_BLOCKS, TUNE_GLDS_TILE, TUNE_SMALLK_TILE, TUNE_X3_RATE_512, TUNE_IN_FUSED,
 TUNE_RESIZE_UP2) = (0, 1, 2, 3, 4, 5)


def tune(ctx: Ctx, key: int, value: int) -> int:
    """Set a planner knob (s2v_tune, host-only); returns the previous value."""
    old = ctypes.c_longlong(0)
    check(ctx.lib.s2v_tune(key, value, ctypes.byref(old)), "s2v_tune")
    return old.value


@contextlib.contextmanager
def tuned(ctx: Ctx, key: int, value: int):
    """s2v_tune ``key`` = ``value`` for the launches issued (captured) inside the block (0: unchanged)."""
    if not value:
        yield
        return
    old = tune(ctx, key, value)
    try:
        yield
    finally:
        tune(ctx, key, old)


@contextlib.contextmanager
def x3_grid_cap(ctx: Ctx, blocks: int):
    """s2v_conv_params.grid_cap = ``blocks`` (rounded down to a multiple of 8) for the convs issued on
    ``ctx`` inside the block: a 256x256-tile split-precision conv with more tiles than that runs as
    ``blocks`` persistent blocks (0: one block per tile).  Per context, not process-wide."""
    prev = getattr(ctx, "grid_cap", 0)
    ctx.grid_cap = max(0, int(blocks)) // 8 * 8
    try:
        yield
    finally:
        ctx.grid_cap = prev


def half_chip_blocks(device) -> int:
    """Half the device's CUs, a multiple of 8 (one persistent block per CU on half the chip)."""
    cus = torch.cuda.get_device_properties(torch.device(device)).multi_processor_count
    return max(8, cus // 2 // 8 * 8)


def conv_splits(ctx: Ctx, p) -> int:
    return (p.plan if isinstance(p, ConvLaunch) else _plan(ctx, p))[5]


def layernorm2d(ctx: Ctx, x: NHWC, weight, bias, y: NHWC, *, act=ACT_LRELU, alpha=0.1, pool=False,
                res: NHWC | None = None, eps=1e-5):
    rv = None if res is None else res.v
    _with_ws(ctx, lambda ws: S2V.layernorm2d_(x.v, weight, bias, eps, act, alpha, pool, rv, y.v, ws))
    return y


def instnorm(ctx: Ctx, x: NHWC, y: NHWC, gamma=None, beta=None, *, act=ACT_NONE, alpha=0.0,
             res: NHWC | None = None, eps=1e-5, pad_out: NHWC | None = None):
    """InstanceNorm2d (+ ADAIN: gamma / beta [N, C] row views) + act (+ res).  ``pad_out``
    ([n, h+2, w+2, c] view) also receives F.pad(y, (1, 1, 1, 1), 'reflect')."""
    if pad_out is not None:
        assert (pad_out.n, pad_out.h, pad_out.w, pad_out.c) == (x.n, x.h + 2, x.w + 2, x.c)
    rv, pv = None if res is None else res.v, None if pad_out is None else pad_out.v
    _with_ws(ctx, lambda ws: S2V.instnorm_(x.v, gamma, beta, eps, act, alpha, rv, y.v, pv, ws))
    return y


def adain_params(ctx: Ctx, hid: torch.Tensor, nhidden: int, w2t: torch.Tensor, bias: torch.Tensor, seg: torch.Tensor,
                 out: torch.Tensor):
    S2V.adain_params_(hid, nhidden, w2t, bias, seg, out)
    return out


def modconv_demod(ctx: Ctx, s: torch.Tensor, wsq: torch.Tensor, out: torch.Tensor, *, eps=1e-8, post=1.0):
    """s: [B, cin] view (row stride s.stride(0)), wsq: [cout, cin], out: [B, cout]."""
    S2V.modconv_demod_(s, wsq, out, eps, post)
    return out


class DemodRows:
    """The demodulated layers of one StyleGAN2 decoder as one row table (``s2v::modconv_demod_rows_``):
    ``layers`` = [(s_off, wsq [cout, cin])...] in row order; layer l's demodulation vector is columns
    ``self.r0[l] : self.r0[l] + cout_l`` of the [B, nrows] output."""

    def __init__(self, layers, device):
        rows, ws, r0, w_off, reach = [], [], [], 0, 0
        for s_off, wsq in layers:
            cout, cin = wsq.shape
            r0.append(len(rows))
            rows += [(s_off, cin, w_off + o * cin, 0) for o in range(cout)]
            ws.append(wsq.reshape(-1).float().cpu())
            w_off += cout * cin
            reach = max(reach, s_off + cin)
        assert w_off < 2 ** 31, "demod table: squared weights past int32 offsets"
        self.rows = torch.tensor(rows, dtype=torch.int32).to(device)
        self.wsq = torch.cat(ws).contiguous().to(device)
        self.r0, self.nrows, self.s_reach = r0, len(rows), reach


def modconv_demod_rows(ctx: Ctx, s: torch.Tensor, table: DemodRows, out: torch.Tensor, *, eps=1e-8, post=1.0):
    """s: [B, >= table.s_reach] style bank (unit column stride), out: [B, >= table.nrows]."""
    S2V.modconv_demod_rows_(s, table.rows, table.wsq, out, eps, post, table.s_reach)
    return out


def torch_bilinear_scale(in_size: int, out_size: int, scale_factor=None) -> float:
    """area_pixel_compute_scale (align_corners=False) as PyTorch computes it (float32)."""
    if scale_factor is not None and scale_factor > 0:
        return float(torch.tensor(1.0 / scale_factor, dtype=torch.float32))
    return float(torch.tensor(in_size, dtype=torch.float32) / out_size)


def resize(ctx: Ctx, x: torch.Tensor, x_off: int, x_shape, x_strides, y: torch.Tensor, y_off: int, y_hw, y_strides, *,
           scale_factor=None, mode=0):
    """F.interpolate between strided views (``s2v::resize_``): the view of x starts ``x_off``
    elements into x's data with x_shape = (n, c, ih, iw) and strides (sn, sc, sy, sx) in elements
    (any sign); the same for y with its (oh, ow).  mode 0 bilinear, 1 nearest."""
    n, c, ih, iw = x_shape
    oh, ow = y_hw
    sh = torch_bilinear_scale(ih, oh, scale_factor) if mode == 0 else (
        float(torch.tensor(1.0 / scale_factor, dtype=torch.float32)) if scale_factor else ih / oh)
    sw = torch_bilinear_scale(iw, ow, scale_factor) if mode == 0 else (
        float(torch.tensor(1.0 / scale_factor, dtype=torch.float32)) if scale_factor else iw / ow)
    S2V.resize_(x, x_off, [n, c, ih, iw], list(x_strides), y, y_off, [n, c, oh, ow], list(y_strides), sh, sw, mode)


def nhwc_strides(v: NHWC):
    return (v.h * v.w * v.cs, 1, v.w * v.cs, v.cs)


def resize_nhwc(ctx: Ctx, x: NHWC, y: NHWC, scale_factor=None, mode=0):
    resize(ctx, x.t, x.coff, (x.n, x.c, x.h, x.w), nhwc_strides(x), y.t, y.coff, (y.h, y.w), nhwc_strides(y),
           scale_factor=scale_factor, mode=mode)
    return y


def nchw_to_nhwc(ctx: Ctx, x: torch.Tensor, y: NHWC, size=None):
    """NCHW device tensor (any strides) -> NHWC view, optionally bilinear-resized to y's size."""
    _require_cuda(x, "nchw_to_nhwc")
    resize(ctx, x, 0, tuple(x.shape), x.stride(), y.t, y.coff, (y.h, y.w), nhwc_strides(y))
    return y


def nhwc_to_nchw(ctx: Ctx, x: NHWC, out: torch.Tensor, crop=(0, 0)):
    """NHWC view (optionally cropped by (top, left) to out's H, W) -> contiguous NCHW tensor."""
    n, c, oh, ow = out.shape
    off = x.coff + (crop[0] * x.w + crop[1]) * x.cs
    resize(ctx, x.t, off, (n, c, oh, ow), nhwc_strides(x), out, 0, (oh, ow), out.stride())
    return out


def torgb_up2(ctx: Ctx, x: NHWC, cw: "ConvW", s: torch.Tensor, skip: NHWC, y: NHWC):
    """ToRGB (1x1 modulated conv to 3 channels, no demodulation, + bias) plus the x2 bilinear
    upsample of ``skip`` in one pass (``s2v::torgb_up2_``, base_blocks.py:536-554).  skip / y carry 4
    channels (the 4th is the upsampled skip's 4th).  s: [B, cin] row view."""
    assert cw.kh == cw.kw == 1 and cw.cout == 3 and x.c == cw.cin, "torgb_up2: a 1x1 conv to 3 channels"
    assert (y.n, y.h, y.w, y.c) == (x.n, x.h, x.w, 4) and (skip.n, 2 * skip.h, 2 * skip.w, skip.c) == (x.n, x.h, x.w, 4)
    S2V.torgb_up2_(x.v, cw.wt, s, cw.shift, skip.v, y.v)
    return y


def row_pack(ctx: Ctx, x: NHWC, y: NHWC, kw: int, pw: int):
    """y[n, h, w, dx * c + ci] = x[n, h, w + dx - pw, ci] (zero outside the row and past kw * c)."""
    S2V.row_pack_(x.v, y.v, kw, pw)
    return y


def pad_reflect(ctx: Ctx, x: NHWC, y: NHWC, pads):
    S2V.pad_reflect_(x.v, y.v, list(pads))
    return y


def row_layernorm(ctx: Ctx, x: torch.Tensor, weight, bias, y: torch.Tensor, eps=1e-5):
    S2V.row_layernorm_(x, weight, bias, eps, y)
    return y


def attention(ctx: Ctx, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, out: torch.Tensor, *, batch, heads,
              tokens, dim_head=64, scale=None):
    """q, k, v, out: [batch*tokens, *] row views (row stride = stride(0)); head h = cols [64h, 64h+64)."""
    scale = dim_head ** -0.5 if scale is None else scale
    S2V.attention_(q, k, v, out, batch, heads, tokens, dim_head, scale)
    return out


def flow_warp(ctx: Ctx, flow: NHWC, src: torch.Tensor, y: NHWC):
    """flow: NHWC view with >= 2 channels (x, y); src: NCHW-strided device tensor."""
    S2V.flow_warp_(flow.v, src, y.v)
    return y


def flow_warp_cat(ctx: Ctx, flow: NHWC, src: torch.Tensor, y: NHWC):
    """y (2C channels) <- [src | warp(src)]: the copy and the warp in one pass (``s2v::flow_warp_cat_``)."""
    S2V.flow_warp_cat_(flow.v, src, y.v)
    return y


def fill(ctx: Ctx, t: torch.Tensor, value: float = 0.0):
    S2V.fill_value_(t, value)
    return t


def pad_cin(w: torch.Tensor, cin: int) -> torch.Tensor:
    """Zero-pad a conv weight [O, I, kh, kw] along I (vectorised 4-channel image layout)."""
    if w.shape[1] >= cin:
        return w
    z = torch.zeros((w.shape[0], cin - w.shape[1]) + tuple(w.shape[2:]), dtype=w.dtype)
    return torch.cat([w, z], 1)


def _i64(v: int) -> int:
    """A 64-bit pattern as the signed int64 a torch op schema carries."""
    v &= 2 ** 64 - 1
    return v - 2 ** 64 if v >= 2 ** 63 else v


def gaussian_noise(ctx: Ctx, out: torch.Tensor, seed: int, offset: int = 0, ctr: torch.Tensor | None = None,
                   shift: int = 40):
    """N(0,1) into ``out``; with a device counter ``ctr`` (int64 [1]) the stream offset advances by
    ctr << shift, read when the kernel runs (fresh draws on every graph replay)."""
    S2V.gaussian_noise_(out, _i64(seed), _i64(offset), ctr, shift)
    return out


class NoiseCounter:
    """Device-side draw counter of an engine's random noise (StyleConv / GFPGAN randomize_noise):
    bumped by a kernel at the start of each forward, so a captured graph draws fresh noise per
    replay.  Created on the first (eager) forward, never inside a capture."""

    def __init__(self):
        self.t = None

    def bump(self, ctx: Ctx) -> torch.Tensor:
        if self.t is None:
            if ctx.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise _lib.S2VError("noise counter must be created by an eager run before graph capture")
            self.t = torch.zeros(1, dtype=torch.int64, device=ctx.device)
        S2V.counter_add_(self.t, 1)
        return self.t


# ----------------------------------------------------------------------------- DFT matrices
_DFT_CACHE = {}


def fourier_matrices(h: int, w: int, device):
    """Real matrices of torch.fft.rfftn / irfftn(s=(h, w)) with norm='ortho' (ffc.py:99, :121).

    D2  [2F, P]: spectrum rows ordered (u*Wf + v)*2 + part (part 0 = real, 1 = imag)
    Iv  [P, 2F]: the inverse (Hermitian c2r) acting on the same row order.
    Built by applying torch.fft (float64) to basis vectors, so they are exactly the reference's
    transforms, including the c2r treatment of the imaginary DC/Nyquist bins."""
    key = (h, w, str(device))
    if key not in _DFT_CACHE:
        P, wf = h * w, w // 2 + 1
        F = h * wf
        eye = torch.eye(P, dtype=torch.float64).reshape(P, h, w)
        spec = torch.fft.rfftn(eye, dim=(-2, -1), norm="ortho").reshape(P, F)      # [P, F] complex
        d2 = torch.stack([spec.real, spec.imag], -1).reshape(P, 2 * F).t()           # [2F, P]
        basis = torch.zeros(2 * F, F, dtype=torch.complex128)
        idx = torch.arange(F)
        basis[2 * idx, idx] = 1.0
        basis[2 * idx + 1, idx] = 1.0j
        iv = torch.fft.irfftn(basis.reshape(2 * F, h, wf), s=(h, w), dim=(-2, -1), norm="ortho")
        iv = iv.reshape(2 * F, P).t()                                                # [P, 2F]
        _DFT_CACHE[key] = (d2.float().contiguous().to(device), iv.float().contiguous().to(device))
    return _DFT_CACHE[key]


# ----------------------------------------------------------------------------- FIR / elementwise
def fir2d(ctx: Ctx, x: NHWC, kernel: torch.Tensor, y: NHWC, *, up=1, down=1, pad0=(0, 0), gain=1.0, bias=None,
          act=ACT_NONE, alpha=0.0, post=1.0):
    """upfirdn2d on NHWC views (pad0 = (pad_y0, pad_x0); the far pads follow from y's size)
    with y = post * act(gain * fir + bias[c])."""
    assert x.n == y.n and x.c == y.c, "fir2d: batch / channel mismatch"
    S2V.fir2d_(x.v, kernel, y.v, up, down, pad0[0], pad0[1], gain, bias, act, alpha, post)
    return y


def eltwise(ctx: Ctx, x: NHWC, y: NHWC, *, a=1.0, mul: NHWC | None = None, add: NHWC | None = None, bias=None,
            act=ACT_NONE, alpha=0.0, post=1.0):
    """y = post * act(x * a * mul + add + bias[c]) over NHWC views of equal n/h/w/c (in place ok)."""
    assert (x.n, x.h, x.w, x.c) == (y.n, y.h, y.w, y.c)
    for v in (mul, add):
        assert v is None or (v.n, v.h, v.w, v.c) == (x.n, x.h, x.w, x.c)
    S2V.eltwise_(x.v, None if mul is None else mul.v, None if add is None else add.v, bias, a, act, alpha, post, y.v)
    return y


# ----------------------------------------------------------------------------- separable FFT
_FFT_TABLES = {}


def fft_tables(h: int, w: int, device):
    """1-D ortho transform matrices for s2v_rfft2 / s2v_irfft2 (include/s2v.h), built by applying
    torch.fft to basis vectors in float64: fw[w][2][Wf] | fh[h][2][u] | ih[u][2][h] | iw[Wf][2][w]."""
    key = (h, w, str(device))
    if key not in _FFT_TABLES:
        wf = w // 2 + 1
        rw = torch.fft.rfft(torch.eye(w, dtype=torch.float64), dim=1, norm="ortho")         # [w, Wf]
        fw = torch.stack([rw.real, rw.imag], 1)                                           # [w, 2, Wf]
        fhc = torch.fft.fft(torch.eye(h, dtype=torch.complex128), dim=1, norm="ortho")      # [h, u]
        fh = torch.stack([fhc.real, fhc.imag], 1)                                         # [h, 2, u]
        ihc = torch.fft.ifft(torch.eye(h, dtype=torch.complex128), dim=1, norm="ortho")     # [u, h]
        ih = torch.stack([ihc.real, ihc.imag], 1)                                         # [u, 2, h]
        eye = torch.eye(wf, dtype=torch.float64)
        cre = torch.fft.irfft(torch.complex(eye, torch.zeros_like(eye)), n=w, dim=1, norm="ortho")   # [v, w]
        cim = torch.fft.irfft(torch.complex(torch.zeros_like(eye), eye), n=w, dim=1, norm="ortho")
        iw = torch.stack([cre, cim], 1)                                                   # [Wf, 2, w]
        t = torch.cat([fw.reshape(-1), fh.reshape(-1), ih.reshape(-1), iw.reshape(-1)]).float().contiguous()
        assert t.numel() == 2 * wf * w + 4 * h * h + 2 * w * wf
        _FFT_TABLES[key] = t.to(device)
    return _FFT_TABLES[key]


def ffc_fused_ok() -> bool:
    """The fused LNet FFC kernels (s2v_ffc_*) cover the split-precision arithmetic; exact f32 runs the
    separate st1 / rfft2 / fu / irfft2 / st2 / instnorm launches."""
    return PRECISION in ("f16x3", "bf16x3")


def ffc_spec_fwd(ctx: Ctx, xg: NHWC, cw: ConvW, tables: torch.Tensor, t1: NHWC, spec: torch.Tensor):
    """t1 = relu(bn1(x_g conv1)), spec = rfftn(t1, ortho) in one launch (s2v_ffc_spec_fwd): ffc.py:98-104,
    :158-160 (SpectralTransform.conv1 + FourierUnit's rfftn)."""
    prec = prec_code()
    xs, flag = _range(ctx, cw, xg, prec)
    S2V.ffc_spec_fwd_(xg.v, cw.wt_x3(ctx, prec), cw.split_scale(prec), xs, cw.scale, cw.shift, tables, t1.v, spec,
                      flag, prec)
    return t1, spec


def ffc_spec_inv(ctx: Ctx, spec: torch.Tensor, cw: ConvW, tables: torch.Tensor, t1: NHWC, u: NHWC):
    """u = irfftn(relu(bn_fu(spec conv_fu)), ortho) + t1 in one launch (s2v_ffc_spec_inv): ffc.py:106-126,
    :162 (FourierUnit conv + irfftn, SpectralTransform's x + fu(x))."""
    prec = prec_code()
    b, f, c2 = spec.shape
    xs, flag = _range(ctx, cw, NHWC(spec.view(b, f, 1, c2)), prec)
    S2V.ffc_spec_inv_(spec, cw.wt_x3(ctx, prec), cw.split_scale(prec), xs, cw.scale, cw.shift, tables, t1.v, u.v, flag,
                      prec)
    return u


def ffc_norm(ctx: Ctx, y: NHWC, u: NHWC, cw: ConvW, out: NHWC, gamma=None, beta=None, *, act=ACT_NONE, alpha=0.0,
             res: NHWC | None = None, eps=1e-5, pad_out: NHWC | None = None):
    """out = act(IN([y_l | y_g + u conv2]) (1 + gamma) + beta) (+ res) (s2v_ffc_norm): SpectralTransform.conv2
    (ffc.py:164), FFC's out_xg sum (ffc.py:225-229) and ADAIN + LeakyReLU (base_blocks.py:143-157, :376-386)
    in one launch; ``pad_out`` also receives F.pad(out, 1, 'reflect')."""
    prec = prec_code()
    xs, flag = _range(ctx, cw, u, prec)
    S2V.ffc_norm_(y.v, u.v, cw.wt_x3(ctx, prec), cw.split_scale(prec), xs, gamma, beta, eps, act, alpha,
                  None if res is None else res.v, out.v, None if pad_out is None else pad_out.v, flag, prec)
    return out


def rfft2(ctx: Ctx, x: NHWC, tables: torch.Tensor, spec: torch.Tensor):
    """x NHWC [n,h,w,C] -> spec [n, h*(w//2+1), 2C] (channel = part*C + c), rfftn ortho."""
    S2V.rfft2_(x.v, tables, spec)
    return spec


def irfft2(ctx: Ctx, spec: torch.Tensor, tables: torch.Tensor, y: NHWC, res: NHWC | None = None):
    """spec [n, F, >=2C] -> y NHWC = irfftn(spec, s=(h, w), ortho) (+ res)."""
    S2V.irfft2_(spec, tables, None if res is None else res.v, y.v)
    return y
