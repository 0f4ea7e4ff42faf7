"""Portable deterministic synthetic checkpoints.

The reference's checkpoints (LNet.pth / ENet.pth / DNet.pt, GFPGANv1.4, GPEN-BFR-512) are not
distributed with it (reference README.md:79), and there is no network.  Every parity fixture,
test, smoke run and benchmark therefore uses weights produced by this module: a counter hash
(splitmix64 of (crc32(key), element index)) turned into uniform values and scaled per parameter
kind.  It depends only on numpy integer arithmetic, so the container that wrote the golden
fixtures and the GPU box regenerate bit-identical weight_orig / bias / BN tensors.

Spectral-norm buffers (``weight_u`` / ``weight_v``) are the leading singular vectors of the
``weight_orig`` matrix (float64 SVD), i.e. what a converged power iteration stores, so the eval
forward W / (u^T W v) (torch.nn.utils.spectral_norm, used at reference models/base_blocks.py:72-76)
divides by the top singular value.
"""
from __future__ import annotations

import re
import zlib

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def hash_uniform(key: str, n: int) -> np.ndarray:
    """n float64 values in [-1, 1) from splitmix64(crc32(key) * golden + i)."""
    seed = np.uint64(zlib.crc32(key.encode("utf-8")))
    with np.errstate(over="ignore"):
        z = np.arange(n, dtype=np.uint64) + seed * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    return 2.0 * u - 1.0


_NOISE_WEIGHT = re.compile(r"(^|\.)(style_convs\.\d+|style_conv1)\.weight$")
_TRANSPOSED = ("conv_s.weight", "conv_1.weight")  # DNet ADAINDecoderBlock ConvTranspose2d


def _is_norm_weight(key: str, shape) -> bool:
    if len(shape) == 1:
        return True
    return len(shape) == 3 and shape[1] == 1 and shape[2] == 1  # LayerNorm2d [C,1,1]


def synth_tensor(key: str, shape, gain: float = 1.3, noise_weight: float = 0.0) -> np.ndarray:
    """Synthetic value for one state_dict entry (float32, or int64 for num_batches_tracked)."""
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    u = hash_uniform(key, n).reshape(shape)
    if ".noises.noise" in key or key.endswith("constant_input.weight"):
        return (u * np.sqrt(3.0)).astype(np.float32)     # torch.randn buffers / parameters: unit variance
    if leaf == "running_mean":
        v = 0.1 * u
    elif leaf == "running_var":
        v = 1.0 + 0.25 * u
    elif leaf == "bias":
        v = 1.0 + 0.1 * u if key.endswith("modulation.bias") else 0.1 * u
    elif leaf in ("weight", "weight_orig"):
        if _NOISE_WEIGHT.search(key):
            v = np.full(shape, noise_weight)
        elif _is_norm_weight(key, shape):
            v = 1.0 + 0.1 * u
        else:
            if len(shape) == 5:            # ModulatedConv2d weight [1, out, in, k, k]
                fan = int(np.prod(shape[2:]))
            elif key.endswith(_TRANSPOSED) and len(shape) == 4:
                fan = shape[0] * shape[2] * shape[3] // 4   # ConvTranspose2d stride 2: [in, out, k, k]
            else:
                fan = int(np.prod(shape[1:]))
            v = u * (np.sqrt(3.0) * gain / np.sqrt(max(fan, 1)))
    else:
        v = 0.1 * u
    return v.astype(np.float32)


def blur_kernel(factor: int = 1) -> np.ndarray:
    """gpen_model.py:26-35 make_kernel([1, 3, 3, 1]) (x factor^2 for the upsampling blurs)."""
    k = np.array([1.0, 3.0, 3.0, 1.0])
    k = np.outer(k, k)
    return (k / k.sum() * factor ** 2).astype(np.float32)


_GPEN_STYLE_MLP = re.compile(r"^generator\.style\.\d+\.weight$")


def synth_equal_tensor(key: str, shape, noise_weight: float = 0.0, lr_mlp: float = 0.01) -> np.ndarray:
    """GPEN (equalized learning rate, gpen_model.py:94-167): parameters are stored as N(0,1)
    draws (divided by lr_mul for the style MLP) and scaled at run time, so synthetic weights are
    unit-variance uniforms; blur kernels are the fixed make_kernel buffers."""
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "kernel":
        return blur_kernel(2 if key.endswith(("conv.blur.kernel", "upsample.kernel")) else 1).reshape(shape)
    if key.endswith("noise.weight"):
        return np.full(shape, noise_weight, dtype=np.float32)
    u = hash_uniform(key, n).reshape(shape)
    if leaf == "bias":
        v = 1.0 + 0.1 * u if key.endswith("modulation.bias") else 0.1 * u
    elif _GPEN_STYLE_MLP.match(key):
        v = u * np.sqrt(3.0) / lr_mlp
    else:
        v = u * np.sqrt(3.0)
    return v.astype(np.float32)


def synth_equal_state_dict(shapes: dict, noise_weight: float = 0.0) -> dict:
    return {k: synth_equal_tensor(k, s, noise_weight) for k, s in shapes.items()}


def synth_state_dict(shapes: dict, gain: float = 1.3, noise_weight: float = 0.0) -> dict:
    """{key: shape} -> {key: np.ndarray}; spectral-norm u/v derived from weight_orig."""
    out = {}
    for key, shape in shapes.items():
        if key.endswith(("weight_u", "weight_v")):
            continue
        out[key] = synth_tensor(key, shape, gain, noise_weight)
    for key, shape in shapes.items():
        if not key.endswith("weight_u"):
            continue
        base = key[: -len("weight_u")]
        w = out[base + "weight_orig"].astype(np.float64)
        # every spectral-normed layer on the path is a Conv2d (dim 0); LNet.py:89 use_spect=True
        mat = w.reshape(w.shape[0], -1)
        uu, _, vt = np.linalg.svd(mat, full_matrices=False)
        u0, v0 = uu[:, 0], vt[0]
        if u0.sum() < 0:                   # fix the SVD sign so the fixture is unambiguous
            u0, v0 = -u0, -v0
        out[key] = u0.astype(np.float32)
        out[base + "weight_v"] = v0.astype(np.float32)
    return out


def synth_torch_state_dict(module, gain: float = 1.3, noise_weight: float = 0.0, equal: bool = False):
    """Synthetic state_dict for any module whose keys follow the reference layout
    (``equal``: the GPEN equalized-learning-rate scheme)."""
    import torch
    shapes = {k: tuple(v.shape) for k, v in module.state_dict().items()}
    sd = synth_equal_state_dict(shapes, noise_weight) if equal else synth_state_dict(shapes, gain, noise_weight)
    return {k: torch.from_numpy(v) for k, v in sd.items()}


# Enhancer presets (shared by the golden generator, tests and benchmarks).  GFPGAN uses gain 1.0:
# its SFT conditions multiply the decoder features level after level, and at 1.3 the synthetic
# activations grow to ~1e14 by the 512 output; at 1.0 they stay O(1..10) like a trained model's.
GFPGAN_SYNTH = dict(gain=1.0, noise_weight=0.1)
GPEN_SYNTH = dict(noise_weight=0.1, equal=True)
# ParseNet: 18 residual blocks add their branch to the identity level after level; gain 1.0 keeps
# the synthetic logits O(1..10) so the argmax is not decided by fp32 rounding
PARSENET_SYNTH = dict(gain=1.0)
# RRDBNet (RealESRNet): 69 dense blocks, each added back at 0.2; gain 1.0 like ParseNet
RRDB_SYNTH = dict(gain=1.0)
# RetinaFace-R50: 16 bottlenecks add onto the identity; gain 1.0 keeps the features O(1..10)
RETINA_SYNTH = dict(gain=1.0)


# ----------------------------------------------------------------------------- inputs
def hash_array(key: str, shape, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """Deterministic float32 array uniform in [lo, hi) (portable: no RNG state)."""
    n = int(np.prod(shape))
    u = (hash_uniform(key, n) + 1.0) * 0.5
    return (lo + (hi - lo) * u).reshape(shape).astype(np.float32)


def lipsync_inputs(tag: str, batch: int, size: int):
    """(mel [B,1,80,16] in [-4,4), face [B,6,S,S] in [0,1) with the lower half of the masked
    crop zeroed as datagen does (inference.py:397-398), gt [B,3,S,S] = the reference half)."""
    mel = hash_array(f"{tag}.mel", (batch, 1, 80, 16), -4.0, 4.0)
    face = hash_array(f"{tag}.face", (batch, 6, size, size), 0.0, 1.0)
    face[:, :3, size // 2:, :] = 0.0
    gt = face[:, 3:].copy()
    return mel, face, gt


def face_inputs(tag: str, batch: int, size: int = 512):
    """Enhancer input faces [B,3,S,S] in [-1,1) (gfpgan/utils.py:115-117 normalisation)."""
    return hash_array(f"{tag}.face512", (batch, 3, size, size), -1.0, 1.0)


def dnet_inputs(tag: str, batch: int, size: int):
    """(src [B,3,S,S] in [-1,1), coeff [B,73,26] ~ U(-1.5,1.5))."""
    src = hash_array(f"{tag}.src", (batch, 3, size, size), -1.0, 1.0)
    coeff = hash_array(f"{tag}.coeff", (batch, 73, 26), -1.5, 1.5)
    return src, coeff


def sr_frame(tag: str, batch: int, h: int, w: int) -> np.ndarray:
    """uint8 HWC BGR frames [B,H,W,3] (RealESRNet.process input, real_esrnet.py:99-101)."""
    return np.floor(hash_array(f"{tag}.frame", (batch, h, w, 3), 0.0, 256.0)).clip(0, 255).astype(np.uint8)


def probe_indices(n: int, count: int = 2048, key: str = "probe") -> np.ndarray:
    """Fixed pseudo-random flat indices used to pin large tensors by a sample of values."""
    u = (hash_uniform(key, count) + 1.0) * 0.5
    return np.unique(np.minimum((u * n).astype(np.int64), n - 1))
