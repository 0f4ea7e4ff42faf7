"""Shared test helpers: synthetic reference-layout state dicts and comparison utilities."""
import functools

import numpy as np
import torch

import s2v_import  # noqa: F401
from s2v_amd import synth
from s2v_amd.models import arch


GFPGAN_KW = dict(out_size=512, num_style_feat=512, channel_multiplier=2, decoder_load_path=None, fix_decoder=False,
                 num_mlp=8, input_is_latent=True, different_w=True, narrow=1, sft_half=True)   # gfpgan/utils.py:40-50


@functools.lru_cache(maxsize=None)
def synth_sd(net: str):
    """Synthetic state_dict (CPU tensors) in the reference layout for
    'lnet'|'enet'|'dnet'|'gfpgan'|'gpen'."""
    from s2v_amd.models import enhancer_arch as ea
    if net == "gfpgan":
        return synth.synth_torch_state_dict(ea.GFPGANv1CleanParams(**GFPGAN_KW), **synth.GFPGAN_SYNTH)
    if net == "gpen":
        return synth.synth_torch_state_dict(ea.FullGeneratorParams(512, 512, 8, 2), **synth.GPEN_SYNTH)
    if net == "gpen2048":             # GPEN-BFR-2048, the CLI's enhancer face GAN (inference.py:228-231)
        return synth.synth_torch_state_dict(ea.FullGeneratorParams(2048, 512, 8, 2), **synth.GPEN_SYNTH)
    mod = {"lnet": lambda: arch.LNetParams(), "enet": lambda: arch.ENetParams(lnet=arch.LNetParams()),
           "dnet": lambda: arch.DNetParams()}[net]()
    return synth.synth_torch_state_dict(mod)


@functools.lru_cache(maxsize=None)
def parsenet_sd(size: int = 512):
    """Synthetic ParseNet state_dict at the FaceParse configuration for ``size`` (face_parsing.py:34)."""
    from s2v_amd.models.parse_arch import ParseNetParams, face_parse_net
    return synth.synth_torch_state_dict(ParseNetParams(**face_parse_net(size)), **synth.PARSENET_SYNTH)


# tests/golden/make_golden.py RRDB_FORWARD / RRDB_PROCESS (kept in sync; the GPU box has no reference)
RRDB_FORWARD = (("s2", 2, (1, 3, 32, 28)), ("s4", 4, (1, 3, 12, 16)), ("s1", 1, (2, 3, 16, 24)))
RRDB_PROCESS = (("p2", 2, 27, 31, 0, 10), ("p2t", 2, 30, 26, 16, 4), ("p4", 4, 13, 11, 0, 10))


@functools.lru_cache(maxsize=None)
def rrdb_sd(scale: int = 2, num_feat: int = 32):
    """Synthetic RRDBNet state_dict at the RealESRNet configuration (real_esrnet.py:22)."""
    from s2v_amd.models.sr_arch import RRDBNetParams
    return synth.synth_torch_state_dict(RRDBNetParams(3, 3, scale=scale, num_feat=num_feat, num_block=23,
                                                      num_grow_ch=32), **synth.RRDB_SYNTH)


def max_abs(a, b):
    a = a.detach().cpu().double().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if isinstance(b, torch.Tensor) else np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    d = np.abs(a - b)
    return float(d.max()), float(d.mean())


def check_probe(t, g, name, atol, rtol=0.0):
    flat = t.detach().cpu().reshape(-1).double().numpy()
    idx, val = g[f"{name}_idx"], g[f"{name}_val"].astype(np.float64)
    got = flat[idx]
    err = np.abs(got - val)
    lim = atol + rtol * np.abs(val)
    assert (err <= lim).all(), f"{name}: max err {err.max():.3e} (limit {lim.max():.3e})"
    return float(err.max())
