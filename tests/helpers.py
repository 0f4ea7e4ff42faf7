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
    if net == "retinaface":           # RetinaFace-R50 (face_detect/retinaface_detection.py:19-30)
        from s2v_amd.models.retinaface_arch import RetinaFaceParams
        return synth.synth_torch_state_dict(RetinaFaceParams(), **synth.RETINA_SYNTH)
    if net == "recon":                # face3d ReconNetWrapper('resnet50') (inference_utils.py:261-267)
        from s2v_amd.models.face3d_arch import ReconNetWrapperParams
        return synth.synth_torch_state_dict(ReconNetWrapperParams(), **synth.RETINA_SYNTH)
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


# ----------------------------------------------------------------------------- face detection
# RetinaFace fixture sizes: image (H, W) of the detection tail case (feature maps ceil(H / 8, 16, 32))
FACE_IMG_HW = (100, 120)
# synthetic 5-point landmark sets (x0..x4, y0..y4: the reshape(2, 5) layout FaceEnhancement passes)
FACE_LANDMARKS = (
    [[430.2, 560.9, 497.0, 440.1, 551.3], [512.5, 508.1, 590.2, 660.4, 655.0]],
    [[100.0, 160.0, 131.0, 108.0, 152.0], [120.0, 124.0, 150.0, 181.0, 184.0]],
    [[812.7, 870.2, 851.9, 800.4, 846.6], [300.1, 321.8, 352.0, 381.7, 399.5]],   # rolled face
    [[30.3, 41.0, 35.2, 31.9, 40.1], [50.7, 50.9, 56.1, 61.5, 61.8]],             # small face
)


def retina_tail_inputs(hw=FACE_IMG_HW):
    """Synthetic backbone features (layer2 / layer3 / layer4 outputs) for the FPN + SSH + heads case."""
    h, w = hw
    sizes = [(-(-h // s), -(-w // s)) for s in (8, 16, 32)]
    return [synth.hash_array(f"golden.retina.f{i}", (1, c, a, b), 0.0, 2.0)
            for i, (c, (a, b)) in enumerate(zip((512, 1024, 2048), sizes))]


def retina_head_outputs(hw=FACE_IMG_HW):
    """Synthetic (loc, conf, landms) for RetinaFaceDetection.detect's post-processing: clusters of
    confident, overlapping anchors so the threshold, the sort and the NMS all act."""
    from oracle.face import prior_box
    pr = prior_box(hw).numpy()
    P = pr.shape[0]
    loc = synth.hash_array("golden.retina.loc", (P, 4), -0.5, 0.5)
    lm = synth.hash_array("golden.retina.lm", (P, 10), -1.0, 1.0)
    u = (synth.hash_array("golden.retina.score", (P,), 0.0, 1.0)).astype(np.float64)
    s = np.where(u > 0.92, 0.9 + 0.1 * (u - 0.92) / 0.08, 0.95 * u)
    conf = np.stack([1.0 - s, s], 1).astype(np.float32)
    return loc, conf, lm


# ----------------------------------------------------------------------------- media fixtures
def write_wav(path, rate=44100, channels=2, seconds=1.0, freq=440.0, amp=0.5):
    """PCM16 .wav with a sine (left) and its half (right), like examples/audio/1.wav's format."""
    import wave
    t = np.arange(int(rate * seconds)) / rate
    left = amp * np.sin(2 * np.pi * freq * t)
    chans = [left, 0.5 * left][:channels]
    pcm = np.clip(np.round(np.stack(chans, 1) * 32767), -32768, 32767).astype("<i2")
    with wave.open(str(path), "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes(pcm.tobytes())
    return path


def write_mp4_header(path, width=320, height=240, frames=30, timescale=12800, duration=15360):
    """A minimal ISO BMFF file with one video track header (tkhd / mdhd / hdlr / stts), no media."""
    import struct

    def box(t, body):
        return struct.pack(">I4s", 8 + len(body), t.encode()) + body
    tkhd = bytes(4) + bytes(20) + bytes(8) + bytes(8) + bytes(36) + struct.pack(">II", width << 16, height << 16)
    mdhd = bytes(4) + bytes(8) + struct.pack(">II", timescale, duration) + bytes(4)
    hdlr = bytes(4) + bytes(4) + b"vide" + bytes(12) + b"VideoHandler\x00"
    stts = bytes(4) + struct.pack(">III", 1, frames, duration // frames)
    stbl = box("stbl", box("stts", stts))
    mdia = box("mdia", box("mdhd", mdhd) + box("hdlr", hdlr) + box("minf", stbl))
    moov = box("moov", box("trak", box("tkhd", tkhd) + mdia))
    with open(path, "wb") as f:
        f.write(box("ftyp", b"isom" + bytes(4)) + moov)
    return path


# ----------------------------------------------------------------------------- 3DMM extraction
FACE3D_HW = (180, 240)
# stand-in for the 5 standard 3D landmarks of BFM's similarity_Lm3D_all.mat (checkpoints/BFM is not
# in the reference tree): eye centres, nose tip, mouth corners in the BFM's y-up frame
FACE3D_LM3D = np.array([[-0.31, 0.29, 0.41], [0.31, 0.29, 0.41], [0.0, 0.0, 0.65], [-0.25, -0.36, 0.44],
                        [0.25, -0.36, 0.44]], np.float64)
# (eye distance px, centre x, centre y, roll deg): mild, 2.5x downscale past the border, 2x upscale
# in a corner, rolled, ~6x downscale; plus one frame with no landmarks (all -1)
FACE3D_CASES = ((60.0, 120.0, 85.0, 0.0), (150.0, 110.0, 95.0, 4.0), (28.0, 32.0, 40.0, -6.0),
                (70.0, 140.0, 100.0, 20.0), (420.0, 120.0, 90.0, 0.0), None)


def face3d_frames(n, hw=FACE3D_HW):
    """Synthetic uint8 RGB frames [n, H, W, 3]."""
    h, w = hw
    return np.floor(synth.hash_array("golden.face3d.frames", (n, h, w, 3), 0.0, 256.0)).astype(np.uint8)


def face3d_landmarks(cases=FACE3D_CASES):
    """68-point (x, y) landmark sets, image coordinates (y down, as FAN writes them): hash noise with
    the seven points extract_5p reads (30, 36, 39, 42, 45, 48, 54) placed as a face."""
    out = []
    for i, c in enumerate(cases):
        if c is None:
            out.append(np.full((68, 2), -1.0, np.float32))
            continue
        d, cx, cy, roll = c
        lm = synth.hash_array(f"golden.face3d.lm{i}", (68, 2), -0.6, 0.6) * d + np.array([cx, cy], np.float32)
        pts = {30: (0.0, 0.05), 36: (-0.7, -0.45), 39: (-0.3, -0.45), 42: (0.3, -0.45), 45: (0.7, -0.45),
               48: (-0.42, 0.62), 54: (0.42, 0.62)}
        a = np.deg2rad(roll)
        for k, (u, v) in pts.items():
            x, y = u * d / 1.0, v * d
            lm[k] = (cx + np.cos(a) * x - np.sin(a) * y, cy + np.sin(a) * x + np.cos(a) * y)
        out.append(lm.astype(np.float32))
    return out


# (w0, h0, w, h, filter) resize cases pinned directly against Pillow: up, down, one axis unchanged,
# both unchanged, bilinear
PIL_RESIZE_CASES = ((37, 29, 61, 45, 3), (90, 70, 23, 31, 3), (40, 33, 40, 70, 3), (40, 33, 17, 33, 3),
                    (50, 40, 50, 40, 3), (45, 38, 70, 19, 2))
