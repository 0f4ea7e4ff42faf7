#!/usr/bin/env python3
"""Per-phase timing of GFPGANer.enhance (s2v_amd.restore; gfpgan/utils.py:97-143) on one synthetic
frame with synthetic weights: the RetinaFace-R50 network and detect_faces(img, 0.97) on the frame
(random weights: the candidate count, hence the host NMS, is not a real frame's), then the composition with a fixed centre face (LMEDS fit,
gray-border warp, GFPGANv1Clean, tensor2img, paste-back).  ms per call, best of --iters.

    python tools/restore_micro.py [--h 720 --w 1280] [--iters 10]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401


class _Rows:
    def __init__(self, rows):
        self.rows = rows

    def detect_faces(self, img, conf_threshold=0.8):
        return self.rows.copy()


def best_ms(fn, iters):
    fn()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=720)
    ap.add_argument("--w", type=int, default=1280)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-detect", action="store_true", help="skip the RetinaFace timing (profiling runs)")
    a = ap.parse_args()
    from helpers import GFPGAN_KW, synth_sd
    from oracle import restore as OR
    from s2v_amd import models, restore
    dev = "cuda"
    H, W = a.h, a.w
    img = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    rf = models.RetinaFace()
    rf.load_state_dict(synth_sd("retinaface"), strict=True)
    det = restore.RetinaFaceDetector(device=dev, net=rf.eval())
    g = models.GFPGANv1Clean(**GFPGAN_KW)
    g.load_state_dict(synth_sd("gfpgan"), strict=True)
    sc = min(H, W) * 0.5 / 512
    p = (OR.FFHQ_TEMPLATE_512 - 256.0) * sc + np.array([W / 2, H / 2])
    rows = np.array([[W / 2 - 200 * sc, H / 2 - 250 * sc, W / 2 + 200 * sc, H / 2 + 250 * sc, 0.999] +
                     list(p.reshape(-1))], np.float32)
    r = restore.GFPGANer(upscale=1, device=dev, net=g.eval(), face_det=_Rows(rows))
    fh = r.face_helper
    res = {}
    if not a.no_detect:
        res["RetinaFace-R50 network (head maps)"] = best_ms(lambda: det.det.head_maps(img), a.iters)
        k = len(det.detect_faces(img, 0.97))
        res[f"detect_faces(img, 0.97) ({k} faces kept)"] = best_ms(lambda: det.detect_faces(img, 0.97), a.iters)

    def align():
        fh.clean_all()
        fh.read_image(img)
        fh.get_face_landmarks_5(only_center_face=True, eye_dist_threshold=5)
        fh.align_warp_face()
    res["landmarks + LMEDS fit + gray-border warp"] = best_ms(align, a.iters)
    align()
    res["img2tensor + GFPGANv1Clean + tensor2img"] = best_ms(lambda: r._restore(fh.cropped_faces), a.iters)
    fh.restored_faces = r._restore(fh.cropped_faces)
    fh.get_inverse_affine(None)
    res["paste_faces_to_input_image"] = best_ms(fh.paste_faces_to_input_image, a.iters)
    res["enhance (fixed face, no detector)"] = best_ms(
        lambda: r.enhance(img, has_aligned=False, only_center_face=True, paste_back=True), a.iters)
    print(f"# GFPGANer.enhance phases on a {W}x{H} uint8 frame, one 512 face, synthetic weights, best of {a.iters}")
    for k, v in res.items():
        print(f"{k:48s} {v:8.2f} ms")


if __name__ == "__main__":
    main()
