"""The inference.py contract on a short clip (BASELINE configs[0]: examples/face/1.mp4 +
examples/audio/1.wav, 8 frames, plumbing).

    python -m s2v_amd.inference --face examples/face/1.mp4 --audio examples/audio/1.wav \
        --max_frames 8 --outfile results/out.npz

Steps (reference file:line in brackets):
  * audio: stdlib ``wave`` PCM -> float32, channels averaged, resampled to 16 kHz
    (audio.load_wav = librosa.load(path, sr=16000), futils/audio.py:10-11) -> mel on the device ->
    16-column windows at 80 / fps columns per frame [inference.py:204-216];
  * video: the MP4 header gives frame size, fps and frame count; there is no video decoder in this
    image (no cv2 / ffmpeg), so the frames are synthetic uint8 BGR frames of that size (SURVEY.md
    §8d allows this), or an .npy [N,H,W,3] uint8 array given as --face;
  * frames truncated to the number of mel windows [inference.py:219-221];
  * the face box: the centred square of --box_frac of the short side (the reference finds it with
    dlib / FAN landmarks, which need packages and weights this image lacks: DESIGN.md §7);
  * 3DMM coefficients: with --checkpoints holding face3d's epoch_20.pth, the built extractor
    (s2v_amd.face3d.Face3DExtractor: align_img + ReconNetWrapper('resnet50'), facing.py:100-130)
    regresses them from the frames with the box-derived 5 landmarks; otherwise they are synthetic;
  * DNet stabilisation of the box crop (trans_image: 256x256, [-1, 1], facing.py:177-191) with the
    coefficient windows, then ENet(LNet) on [masked crop, reference] batches of LNet_batch_size,
    clamp(0, 1) * 255 [inference.py:259-267, :393-399] (s2v_amd.pipeline.LipSyncPipeline);
  * --ref_enhance: Step 5, ``ref_enhancer.process(img, img, face_enhance=False)`` with
    FaceEnhancement(in_size 512, use_sr False) on every stabilised reference before ENet
    [inference.py:224-238] (needs real RetinaFace / ParseNet weights: synthetic ones detect no face,
    and the reference raises on a frame without one);
  * each 384x384 prediction resized into the box and pasted into its frame [inference.py:287-291];
  * --enhance: FaceEnhancement (SR x2, RetinaFace, GPEN-2048, parse-mask paste) on each pasted frame
    against the 2x frame [inference.py:228-231, :317-328]; needs real checkpoints (synthetic
    RetinaFace weights detect no faces, and the reference raises on a frame without one).
Weights come from --checkpoints (LNet.pth / ENet.pth / DNet.pt as models.load_network /
load_DNet read them) or, when absent, from the portable synthetic generator (s2v_amd.synth).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import struct
import sys
import time
import wave

import numpy as np
import torch


# ----------------------------------------------------------------------------- audio
def _pcm_to_float(raw: bytes, width: int) -> np.ndarray:
    if width == 1:
        return (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    if width == 2:
        return np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    if width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        return (np.where(v >= 1 << 23, v - (1 << 24), v)).astype(np.float32) / float(1 << 23)
    if width == 4:
        return np.frombuffer(raw, "<i4").astype(np.float32) / float(1 << 31)
    raise ValueError(f"unsupported PCM sample width {width}")


def resample(x: np.ndarray, sr_in: int, sr_out: int, num_zeros: int = 64, rolloff: float = 0.9475937167399596,
             beta: float = 14.769656459379492) -> np.ndarray:
    """Band-limited (Kaiser-windowed sinc) resampling with librosa 0.9's default 'kaiser_best'
    parameters (resampy: 64 zero crossings, rolloff 0.9476, Kaiser beta 14.77).  resampy's tabulated
    filter is not available here: parity with librosa.load is UNPINNED (the mel front end is)."""
    if sr_in == sr_out:
        return x.astype(np.float32)
    g = math.gcd(sr_in, sr_out)
    up, down = sr_out // g, sr_in // g                      # output k sits at input time k * down / up
    cutoff = rolloff * min(1.0, sr_out / sr_in)
    half = int(math.ceil(num_zeros / cutoff))
    n_out = int(math.ceil(len(x) * sr_out / sr_in))
    taps = np.arange(-half + 1, half + 1)                   # input offsets around floor(t)
    phases = np.arange(up) * down % up / up                 # fractional part of t per phase
    t = taps[None, :] - phases[:, None]                     # [up, 2 half] distance input - t
    win = np.i0(beta * np.sqrt(np.clip(1.0 - (t / (half + 1)) ** 2, 0.0, 1.0))) / np.i0(beta)
    filt = (cutoff * np.sinc(cutoff * t) * win).astype(np.float64)
    xp = np.concatenate([np.zeros(half, np.float64), x.astype(np.float64), np.zeros(2 * half + 1, np.float64)])
    out = np.empty(n_out, np.float64)
    k = np.arange(n_out)
    base = (k * down) // up
    ph = k % up
    for s in range(0, n_out, 8192):
        e = min(n_out, s + 8192)
        idx = base[s:e, None] + half + taps[None, :]
        out[s:e] = np.einsum("ij,ij->i", xp[idx], filt[ph[s:e]])
    return out.astype(np.float32)


def load_wav(path: str, sr: int = 16000) -> np.ndarray:
    """librosa.load(path, sr=sr) for PCM .wav files: float32 mono (channels averaged) at ``sr``."""
    with wave.open(path, "rb") as w:
        ch, width, rate, n = w.getnchannels(), w.getsampwidth(), w.getframerate(), w.getnframes()
        raw = w.readframes(n)
    x = _pcm_to_float(raw, width).reshape(-1, ch).mean(axis=1)
    return resample(x, rate, sr)


# ----------------------------------------------------------------------------- video header
def mp4_video_info(path: str) -> dict:
    """Width, height, frame count and fps of the first video track of an MP4 (ISO BMFF boxes:
    tkhd, mdhd, hdlr, stts) — enough to size synthetic frames when no decoder exists."""
    with open(path, "rb") as f:
        data = f.read()
    tracks = []

    def walk(off, end, cur):
        while off + 8 <= end:
            size, typ = struct.unpack(">I4s", data[off:off + 8])
            hdr = 8
            if size == 1:
                size, hdr = struct.unpack(">Q", data[off + 8:off + 16])[0], 16
            elif size == 0:
                size = end - off
            if size < hdr:
                break
            body = data[off + hdr: off + size]
            t = typ.decode("latin1")
            if t == "trak":
                tr = {}
                tracks.append(tr)
                walk(off + hdr, off + size, tr)
            elif t in ("moov", "mdia", "minf", "stbl"):
                walk(off + hdr, off + size, cur)
            elif t == "tkhd" and cur is not None:
                v = body[0]
                o = 4 + (32 if v == 1 else 20) + 8 + 8 + 36
                cur["width"], cur["height"] = (struct.unpack(">I", body[o + k: o + k + 4])[0] / 65536.0 for k in (0, 4))
            elif t == "mdhd" and cur is not None:
                v = body[0]
                if v == 1:
                    cur["timescale"], cur["duration"] = struct.unpack(">IQ", body[20:32])
                else:
                    cur["timescale"], cur["duration"] = struct.unpack(">II", body[12:20])
            elif t == "hdlr" and cur is not None:
                cur["handler"] = body[8:12].decode("latin1")
            elif t == "stts" and cur is not None:
                n = struct.unpack(">I", body[4:8])[0]
                cur["frames"] = sum(struct.unpack(">I", body[8 + 8 * i: 12 + 8 * i])[0] for i in range(n))
            off += size

    walk(0, len(data), None)
    for tr in tracks:
        if tr.get("handler") == "vide":
            fps = tr["frames"] * tr["timescale"] / tr["duration"] if tr.get("duration") else 25.0
            return {"width": int(round(tr["width"])), "height": int(round(tr["height"])), "frames": tr["frames"],
                    "fps": fps}
    raise ValueError(f"{path}: no video track found")


# ----------------------------------------------------------------------------- runner
def _weights(ckpt_dir):
    from . import models, synth
    from .models import arch
    names = {k: os.path.join(ckpt_dir or "", f) for k, f in (("LNet", "LNet.pth"), ("ENet", "ENet.pth"),
                                                              ("DNet", "DNet.pt"))}
    if ckpt_dir and all(os.path.exists(p) for p in names.values()):
        args = argparse.Namespace(LNet_path=names["LNet"], ENet_path=names["ENet"], DNet_path=names["DNet"])
        return models.load_network(args), models.load_DNet(args), "checkpoints"
    enet = models.ENet(lnet=models.LNet())
    enet.load_state_dict(synth.synth_torch_state_dict(arch.ENetParams(lnet=arch.LNetParams())), strict=True)
    dnet = models.DNet()
    dnet.load_state_dict(synth.synth_torch_state_dict(arch.DNetParams()), strict=True)
    return enet.eval(), dnet.eval(), "synthetic"


def _frames(face: str, max_frames: int):
    from . import synth
    if face.endswith(".npy"):
        fr = np.load(face, allow_pickle=False)
        if fr.dtype != np.uint8 or fr.ndim != 4 or fr.shape[3] != 3:
            raise ValueError("--face .npy must hold uint8 [N,H,W,3] BGR frames")
        return fr[:max_frames], 25.0, "npy"
    info = mp4_video_info(face)
    n = min(info["frames"], max_frames)
    return synth.sr_frame(f"inference.{os.path.basename(face)}", n, info["height"], info["width"]), info["fps"], \
        f"synthetic {info['width']}x{info['height']} (no decoder; {info['frames']} frames in the file)"


# face3d's 5-point 3D reference when BFM/similarity_Lm3D_all.mat is absent (stated stand-in, the
# layout of lm3d_from_68: eyes, nose tip, mouth corners)
LM3D_STANDIN = np.array([[-0.31, 0.29, 0.41], [0.31, 0.29, 0.41], [0.0, 0.0, 0.65], [-0.25, -0.36, 0.44],
                         [0.25, -0.36, 0.44]])


def _semantic(frames_bgr: torch.Tensor, ckpt_dir, dev):
    """facing.py:100-130 face_3dmm_extraction on the frames: ReconNetWrapper('resnet50') from
    face3d_pretrain_epoch_20.pth (synthetic weights without it), the reference's no-landmark path
    (all -1 landmarks -> lm3d positions, facing.py:110-116) since FAN is absent -> [n, 262]."""
    from . import face3d, models, synth
    from .models.face3d_arch import ReconNetWrapperParams
    path = os.path.join(ckpt_dir or "", "face3d_pretrain_epoch_20.pth")
    if ckpt_dir and os.path.exists(path):
        net = models.load_face3d_net(path, dev)
        kind = "checkpoint"
    else:
        net = models.ReconNetWrapper()
        net.load_state_dict(synth.synth_torch_state_dict(ReconNetWrapperParams(), **synth.RETINA_SYNTH))
        net = net.eval()
        kind = "synthetic"
    bfm = os.path.join(ckpt_dir or "", "BFM")
    lm3d = face3d.load_lm3d(bfm) if os.path.exists(os.path.join(bfm, "similarity_Lm3D_all.mat")) else LM3D_STANDIN
    n = frames_bgr.shape[0]
    rgb = frames_bgr[..., [2, 1, 0]].contiguous()                               # facing.py reads RGB PIL frames
    ext = face3d.Face3DExtractor(net, lm3d, dev)
    return ext.face_3dmm_extraction(rgb, np.full((n, 68, 2), -1.0, np.float32)), kind


def _ref_enhancer(ckpt_dir, dev):
    """inference.py:224-226: FaceEnhancement(in_size=512, channel_multiplier=2, narrow=1, sr_scale=4,
    model='GPEN-BFR-512', use_sr=False) as a hook on the stabilised uint8 RGB references."""
    from . import face as faces
    enh = faces.FaceEnhancement(base_dir=ckpt_dir or "checkpoints", in_size=512, channel_multiplier=2, narrow=1,
                                sr_scale=4, model="GPEN-BFR-512", use_sr=False, device=dev)
    return reference_hook(enh)


def reference_hook(enh):
    """Step 5 (inference.py:234-238) as a LipSyncPipeline ref hook: each uint8 RGB [3, h, w] reference
    -> BGR HWC -> ``enh.process_device(img, img, face_enhance=False, possion_blending=False)`` -> back."""
    def hook(ref_u8: torch.Tensor) -> torch.Tensor:
        out = torch.empty_like(ref_u8)
        for i in range(ref_u8.shape[0]):
            bgr = ref_u8[i].flip(0).permute(1, 2, 0).contiguous()
            img = enh.process_device(bgr, bgr, face_enhance=False, possion_blending=False)[0]
            out[i] = img.permute(2, 0, 1).flip(0)
        return out
    return hook


def run(face: str, audio_path: str, max_frames: int = 8, batch: int = 16, box_frac: float = 0.6,
        ckpt_dir: str | None = None, enhance: bool = False, device: str = "cuda", ref_enhance: bool = False,
        ref_hook=None, restore: bool = True, restorer=None, enhancer=None):
    """-> dict(frames uint8 [n,H,W,3] device, preds uint8 [n,3,384,384], meta).  ``ref_enhance``:
    Step 5 with FaceEnhancement-512 (``ref_hook``: any callable on uint8 [b,3,h,w] references).
    ``enhance``: the per-frame tail of inference.py:296-330 on the pasted frames -> ``enhanced``
    uint8 [n,2H,2W,3]: GFPGANer.enhance(ff, only_center_face=True) (``restore``; restore.GFPGANer,
    :300-301), the FaceParse mouth mask + 10-level Laplacian blend (post.MouthBlend, :302-313), then
    FaceEnhancement-2048 with SR x2 on the 2x frame (:326-327).  ``restorer`` / ``enhancer``: given
    objects (else built from ``ckpt_dir`` as the reference builds them)."""
    from . import audio, pipeline, post, synth
    dev = torch.device(device)
    t0 = time.time()
    frames_np, fps, src_kind = _frames(face, max_frames)
    wav = load_wav(audio_path, 16000)
    mel = audio.melspectrogram(torch.from_numpy(wav).to(dev))
    chunks = audio.mel_chunks(mel, fps=fps)
    n = min(len(frames_np), chunks.shape[0])                                        # inference.py:219-221
    frames = torch.from_numpy(np.ascontiguousarray(frames_np[:n])).to(dev)
    H, W = frames.shape[1:3]
    side = int(min(H, W) * box_frac)
    y1, x1 = (H - side) // 2, (W - side) // 2
    y2, x2 = y1 + side, x1 + side
    enet, dnet, wkind = _weights(ckpt_dir)
    # DNet source: trans_image of the box crop (256x256, ToTensor + Normalize(0.5, 0.5), RGB)
    crops = torch.empty((n, 256, 256, 3), dtype=torch.uint8, device=dev)
    for i in range(n):
        post.resize_linear(frames[i, y1:y2, x1:x2], (256, 256), out=crops[i])
    src = torch.empty((n, 3, 256, 256), device=dev)
    ctx = post._ctx(dev)
    from ._lib import check
    check(ctx.lib.s2v_u8_to_gan(crops.data_ptr(), n, 256, 256, src.data_ptr(), ctx.stream), "s2v_u8_to_gan")
    semantic, skind = _semantic(frames, ckpt_dir, dev)                             # facing.py:100-130
    expression = synth.hash_array("inference.expression", (64,), -1.0, 1.0)        # expression.mat is absent
    coeffs = torch.from_numpy(pipeline.dnet_coefficients(semantic, expression, False, 0, n)).to(dev)
    if ref_enhance and ref_hook is None:
        ref_hook = _ref_enhancer(ckpt_dir, dev)
    pipe = pipeline.LipSyncPipeline(dnet, enet, device=dev, batch=batch, graph=False, ref_hook=ref_hook)
    preds = pipe.run(chunks[:n], src, coeffs)                                       # [n,3,384,384] uint8
    out = frames.clone()
    hwc = preds.permute(0, 2, 3, 1).contiguous()
    for i in range(n):                                                              # inference.py:287-291
        post.resize_linear(hwc[i], (x2 - x1, y2 - y1), out=out[i, y1:y2, x1:x2])
    enhanced = None
    if enhance:
        from . import face as faces
        base = ckpt_dir or "checkpoints"
        enh = enhancer or faces.FaceEnhancement(base_dir=base, in_size=2048, channel_multiplier=2, narrow=1,
                                                sr_scale=2, sr_model=None, model="GPEN-BFR-2048", use_sr=True,
                                                device=device)                       # inference.py:228-231
        if restore and restorer is None:
            from .restore import GFPGANer
            restorer = GFPGANer(model_path=os.path.join(base, "GFPGANv1.4.pth"), upscale=1, arch="clean",
                                channel_multiplier=2, bg_upsampler=None, device=device, base_dir=base)   # :255-256
        mouth = post.MouthBlend(enh.faceparser)
        box = (y1, y2, x1, x2)
        enhanced = []
        for i in range(n):
            pp = out[i]
            if restore:
                _, _, restored_img = restorer.enhance(pp, has_aligned=False, only_center_face=True,
                                                      paste_back=True)                  # inference.py:300-301
                pp = mouth.run(restored_img, pp, box)                                   # :302-313
            big = post.resize_linear(frames[i], (2 * W, 2 * H))                      # tmp_xf (inference.py:326)
            enhanced.append(enh.process_device(pp, big, bbox=box, face_enhance=True, possion_blending=True)[0])
        enhanced = torch.stack(enhanced)
    torch.cuda.synchronize(dev)
    meta = {"frames": n, "frame_hw": [int(H), int(W)], "fps": fps, "video": src_kind, "weights": wkind,
            "mel_cols": int(mel.shape[1]), "mel_windows": int(chunks.shape[0]), "wav_samples_16k": int(len(wav)),
            "box": [y1, y2, x1, x2], "semantic": skind, "ref_enhance": ref_hook is not None,
            "restore": bool(enhance and restore),
            "seconds": round(time.time() - t0, 3)}
    return {"frames": out, "preds": preds, "enhanced": enhanced, "meta": meta}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--face", required=True, help="MP4 (header read; synthetic frames) or uint8 [N,H,W,3] .npy")
    ap.add_argument("--audio", required=True, help="PCM .wav")
    ap.add_argument("--outfile", default="results/inference_frames.npz")
    ap.add_argument("--max_frames", type=int, default=8)
    ap.add_argument("--LNet_batch_size", type=int, default=16)
    ap.add_argument("--box_frac", type=float, default=0.6)
    ap.add_argument("--checkpoints", default=None)
    ap.add_argument("--enhance", action="store_true")
    ap.add_argument("--no_restore", action="store_true", help="with --enhance: skip GFPGANer + the mouth blend")
    ap.add_argument("--ref_enhance", action="store_true", help="Step 5: FaceEnhancement-512 on the references")
    a = ap.parse_args(argv)
    r = run(a.face, a.audio, a.max_frames, a.LNet_batch_size, a.box_frac, a.checkpoints, a.enhance,
            ref_enhance=a.ref_enhance, restore=not a.no_restore)
    os.makedirs(os.path.dirname(os.path.abspath(a.outfile)), exist_ok=True)
    arrays = {"frames": r["frames"].cpu().numpy(), "preds": r["preds"].cpu().numpy()}
    if r["enhanced"] is not None:
        arrays["enhanced"] = r["enhanced"].cpu().numpy()
    np.savez_compressed(a.outfile, **arrays)
    print(json.dumps(dict(r["meta"], outfile=a.outfile)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
