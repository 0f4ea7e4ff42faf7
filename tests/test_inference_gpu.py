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
