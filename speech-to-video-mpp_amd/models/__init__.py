"""Drop-in model API of the reference's ``models`` package (models/__init__.py, LNet.py,
ENet.py, DNet.py): same class names, constructor arguments, ``state_dict`` keys, forward
signatures and return values; the forward runs on libs2v (HIP, gfx950).

    from s2v_amd.models import LNet, ENet, DNet, load_network, load_DNet
    model = load_network(args)            # ENet(lnet=LNet()) with checkpoints, eval mode
    pred, low = model.cuda()(mel, img, ref)   # inference.py:266

Weights are folded and packed for the device on the first forward (spectral norm, BatchNorm,
modulation layout); call ``refresh()`` after mutating parameters in place.  Inputs must be CUDA
fp32 tensors: there is no CPU path (the checker for CPU is oracle/, test infrastructure).
"""
from __future__ import annotations

import torch

from .. import ops
from ..ops import NHWC
from . import arch


def _fold5(x, dim):
    return torch.cat([x.select(dim, i) for i in range(x.shape[dim])], 0)


def _need_cuda(*ts):
    for t in ts:
        if not (isinstance(t, torch.Tensor) and t.is_cuda):
            raise RuntimeError("s2v_amd models run on the HIP device only: move the module inputs to 'cuda' "
                               "(there is no CPU fallback on the product path)")


class _EngineMixin:
    _engine_cls = None
    _prefix = ""

    def _engine(self, device):
        cache = self.__dict__.setdefault("_s2v_engines", {})
        key = str(device)
        if key not in cache:
            sd = {k: v.detach().to("cpu") for k, v in self.state_dict().items()}
            cache[key] = (self._build_engine(sd, device), ops.Ctx(device))
        return cache[key]

    def refresh(self):
        self.__dict__.pop("_s2v_engines", None)
        return self

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self.refresh()
        return super().load_state_dict(state_dict, strict=strict, assign=assign)


class LNet(_EngineMixin, arch.LNetParams):
    """models/LNet.py:80-139."""

    def _build_engine(self, sd, device):
        from ..engine.lnet import LNetEngine
        return LNetEngine(sd, device)

    @torch.no_grad()
    def forward(self, audio_sequences, face_sequences):
        _need_cuda(audio_sequences, face_sequences)
        b = audio_sequences.size(0)
        five = face_sequences.dim() > 4
        if five:
            audio_sequences = _fold5(audio_sequences, 1)
            face_sequences = _fold5(face_sequences, 2)
        eng, ctx = self._engine(face_sequences.device)
        n, _, h, w = face_sequences.shape
        dev = face_sequences.device
        x6 = NHWC.empty(n, h, w, 6, dev)
        ops.nchw_to_nhwc(ctx, face_sequences.float(), x6)
        lo = NHWC.empty(n, h, w, 3, dev)
        eng.forward(ctx, audio_sequences.float(), x6, lo)
        out = torch.empty((n, 3, h, w), device=dev)
        ops.nhwc_to_nchw(ctx, lo, out)
        if five:
            out = torch.stack(torch.split(out, b, 0), 2)
        return out


class ENet(_EngineMixin, arch.ENetParams):
    """models/ENet.py:8-139; ``lnet`` is held as ``low_res`` like the reference."""

    def __init__(self, num_style_feat=512, lnet=None, concat=False):
        super().__init__(num_style_feat=num_style_feat, lnet=lnet if lnet is not None else LNet(), concat=concat)

    def _build_engine(self, sd, device):
        from ..engine.enet import ENetEngine
        return ENetEngine(sd, device)

    @torch.no_grad()
    def forward(self, audio_sequences, face_sequences, gt_sequences, noises=None):
        _need_cuda(audio_sequences, face_sequences, gt_sequences)
        b = audio_sequences.size(0)
        five = face_sequences.dim() > 4
        if five:
            audio_sequences = _fold5(audio_sequences, 1)
            face_sequences = _fold5(face_sequences, 2)
            gt_sequences = _fold5(gt_sequences, 2)
        eng, ctx = self._engine(face_sequences.device)
        n = face_sequences.shape[0]
        dev = face_sequences.device
        out = torch.empty((n, 3, 384, 384), device=dev)
        low = torch.empty((n, 3, 96, 96), device=dev)
        eng.forward(ctx, audio_sequences.float(), face_sequences.float(), gt_sequences.float(), out, low, noises)
        if five:
            out = torch.stack(torch.split(out, b, 0), 2)
            low = torch.nn.functional.interpolate(low, out.shape[3:])
            low = torch.stack(torch.split(low, b, 0), 2)
        return out, low


class DNet(_EngineMixin, arch.DNetParams):
    """models/DNet.py:13-28."""

    def _build_engine(self, sd, device):
        from ..engine.dnet import DNetEngine
        return DNetEngine(sd, device)

    @torch.no_grad()
    def forward(self, input_image, driving_source, stage=None):
        _need_cuda(input_image, driving_source)
        eng, ctx = self._engine(input_image.device)
        return eng.forward(ctx, input_image.float(), driving_source.float(), stage=stage)


# ----------------------------------------------------------------------------- loaders
def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def load_checkpoint(path, model):
    """models/__init__.py:12-27: ``state_dict`` entry, ``low_res`` keys skipped, ``module.``
    stripped, strict=False; a bare state_dict file is loaded as-is."""
    print("Load checkpoint from: {}".format(path))
    ckpt = _load(path)
    if isinstance(ckpt, dict) and "state_dict" in ckpt and "arcface" not in path:
        sd = {k.replace("module.", ""): v for k, v in ckpt["state_dict"].items() if "low_res" not in k}
        model.load_state_dict(sd, strict=False)
    else:
        model.load_state_dict(ckpt)
    return model


def load_network(args):
    """models/__init__.py:29-35."""
    lnet = load_checkpoint(args.LNet_path, LNet())
    enet = ENet(lnet=lnet)
    return load_checkpoint(args.ENet_path, enet).eval()


def load_DNet(args):
    """models/__init__.py:50-56: DNet weights from ckpt['net_G_ema'], strict=False."""
    dnet = DNet()
    print("Load checkpoint from: {}".format(args.DNet_path))
    ckpt = _load(args.DNet_path)
    dnet.load_state_dict(ckpt["net_G_ema"], strict=False)
    return dnet.eval()


__all__ = ["LNet", "ENet", "DNet", "load_checkpoint", "load_network", "load_DNet"]
