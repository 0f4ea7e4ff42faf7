"""configs[0] runner (s2v_amd.inference, the inference.py:204-291 contract) on the device: 8 frames
of a synthetic clip (MP4 header -> synthetic frames, PCM wav -> mel windows), DNet -> ENet(LNet) ->
uint8 predictions pasted into the frames."""
import numpy as np
import pytest
import torch

import s2v_import  # noqa: F401
from helpers import write_mp4_header, write_wav

pytestmark = pytest.mark.gpu


def test_runner_eight_frames(tmp_path):
    from s2v_amd import inference, post
    mp4 = write_mp4_header(tmp_path / "v.mp4", 320, 240, 40, 12800, 20480)          # 25 fps
    wav = write_wav(tmp_path / "a.wav", rate=44100, channels=2, seconds=1.0)
    r = inference.run(str(mp4), str(wav), max_frames=8)
    m = r["meta"]
    assert m["frames"] == 8 and m["frame_hw"] == [240, 320] and m["mel_windows"] >= 8
    frames, preds = r["frames"], r["preds"]
    assert frames.shape == (8, 240, 320, 3) and preds.shape == (8, 3, 384, 384) and preds.dtype == torch.uint8
    y1, y2, x1, x2 = m["box"]
    src = torch.from_numpy(inference._frames(str(mp4), 8)[0]).cuda()
    outside = torch.ones((240, 320), dtype=torch.bool)
    outside[y1:y2, x1:x2] = False
    assert torch.equal(frames[:, outside], src[:, outside])                   # only the box is replaced
    for i in range(8):                                                        # inference.py:287-291
        exp = post.resize_linear(preds[i].permute(1, 2, 0).contiguous(), (x2 - x1, y2 - y1))
        assert torch.equal(frames[i, y1:y2, x1:x2], exp)
    r2 = inference.run(str(mp4), str(wav), max_frames=8)
    assert torch.equal(r2["preds"], preds)                                   # deterministic (noise weight 0)


def test_runner_cli_writes_npz(tmp_path):
    from s2v_amd import inference
    mp4 = write_mp4_header(tmp_path / "v.mp4", 200, 180, 12, 12800, 6144)
    wav = write_wav(tmp_path / "a.wav", rate=16000, channels=1, seconds=0.5)
    out = tmp_path / "o.npz"
    assert inference.main(["--face", str(mp4), "--audio", str(wav), "--outfile", str(out), "--max_frames", "8"]) == 0
    z = np.load(out)
    assert z["frames"].shape == (8, 180, 200, 3) and z["preds"].shape == (8, 3, 384, 384)


def test_runner_reference_hook_and_semantic(tmp_path):
    """Step 5 wiring (inference.py:234-238): an identity reference hook gives the frames of the run
    without it; the 3DMM coefficients come from the built extractor (facing.py:100-130)."""
    from s2v_amd import inference
    mp4 = write_mp4_header(tmp_path / "v.mp4", 200, 180, 12, 12800, 6144)
    wav = write_wav(tmp_path / "a.wav", rate=16000, channels=1, seconds=0.5)
    a = inference.run(str(mp4), str(wav), max_frames=5, batch=4)
    calls = []

    def ident(ref):
        calls.append(tuple(ref.shape))
        return ref.clone()
    b = inference.run(str(mp4), str(wav), max_frames=5, batch=4, ref_hook=ident)
    assert calls == [(4, 3, 256, 256), (1, 3, 256, 256)] and b["meta"]["ref_enhance"]
    assert torch.equal(a["preds"], b["preds"]) and a["meta"]["semantic"] == "synthetic"


class _Det:
    """Fixed detections: facexlib rows (``rows``) for GFPGANer, (dets, landms) for FaceEnhancement."""

    def __init__(self, rows=None, dets=None, landms=None):
        self.rows, self.dets, self.landms = rows, dets, landms

    def detect_faces(self, img, conf_threshold=0.8):
        return self.rows.copy()

    def detect(self, img):
        return self.dets, self.landms


def test_runner_enhance_tail_restore_mouth_blend_and_enhancer(tmp_path):
    """The per-frame tail of inference.py:296-330 wired in run(enhance=True): GFPGANer.enhance on the
    pasted frame, the mouth-mask Laplacian blend, FaceEnhancement on the 2x frame — equal to composing
    the three by hand; restore=False skips the first two."""
    from helpers import GFPGAN_KW, parsenet_sd, rrdb_sd, synth_sd
    from oracle import restore as OR
    from s2v_amd import face, inference, models, post, restore, sr
    mp4 = write_mp4_header(tmp_path / "v.mp4", 200, 180, 12, 12800, 6144)
    wav = write_wav(tmp_path / "a.wav", rate=16000, channels=1, seconds=0.5)
    g = models.GFPGANv1Clean(**GFPGAN_KW)
    g.load_state_dict(synth_sd("gfpgan"), strict=True)
    p = (OR.FFHQ_TEMPLATE_512 - 256.0) * 0.2 + np.array([100.0, 95.0])
    rows = np.array([[70, 55, 130, 135, 0.999] + list(p.reshape(-1))], np.float32)
    restorer = restore.GFPGANer(upscale=1, device="cuda", net=g.eval(), face_det=_Det(rows=rows),
                                randomize_noise=False)
    gpen = models.FullGenerator(512, 512, 8, 2)
    gpen.load_state_dict(synth_sd("gpen"), strict=True)
    parse = models.ParseNet(**models.parse_arch.face_parse_net(512))
    parse.load_state_dict(parsenet_sd(512), strict=True)
    srnet = models.RRDBNet(3, 3, scale=2, num_feat=32, num_block=23, num_grow_ch=32)
    srnet.load_state_dict(rrdb_sd(2), strict=True)
    dets = np.array([[140, 110, 260, 270, 0.99]], np.float32)
    lms = np.array([[170, 230, 200, 175, 225, 160, 158, 190, 225, 224]], np.float32)
    enh = face.FaceEnhancement(in_size=512, use_sr=True, sr_scale=2, device="cuda",
                               facedetector=_Det(dets=dets, landms=lms),
                               facegan=face.FaceGAN(in_size=512, device="cuda", net=gpen.eval()),
                               faceparser=post.FaceParse(device="cuda", net=parse.eval()),
                               srmodel=sr.RealESRNet(scale=2, device="cuda", net=srnet.eval()))
    r = inference.run(str(mp4), str(wav), max_frames=2, batch=2, enhance=True, restorer=restorer, enhancer=enh)
    assert r["meta"]["restore"] and r["enhanced"].shape == (2, 360, 400, 3)
    y1, y2, x1, x2 = r["meta"]["box"]
    mouth = post.MouthBlend(enh.faceparser)
    src = torch.from_numpy(inference._frames(str(mp4), 2)[0]).cuda()
    for i in range(2):
        ff = r["frames"][i]
        _, restored, img = restorer.enhance(ff, has_aligned=False, only_center_face=True, paste_back=True)
        assert len(restored) == 1 and not torch.equal(img, ff)
        pp = mouth.run(img, ff, (y1, y2, x1, x2))
        big = post.resize_linear(src[i], (400, 360))
        exp = enh.process_device(pp, big, bbox=(y1, y2, x1, x2), face_enhance=True, possion_blending=True)[0]
        assert torch.equal(r["enhanced"][i], exp)
    r2 = inference.run(str(mp4), str(wav), max_frames=2, batch=2, enhance=True, restore=False, enhancer=enh)
    big = post.resize_linear(src[0], (400, 360))
    exp = enh.process_device(r2["frames"][0], big, bbox=(y1, y2, x1, x2), face_enhance=True, possion_blending=True)[0]
    assert not r2["meta"]["restore"] and torch.equal(r2["enhanced"][0], exp)
