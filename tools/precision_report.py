#!/usr/bin/env python3
"""Measured error of the HIP models against the reference goldens (tests/golden) in every conv
arithmetic mode (exact fp32 MFMA, split-fp32 bf16x3 / f16x3).  ENet is also reported on the
clamp(0, 1) output the caller consumes (inference.py:267) and on the B=16 bench batch against the
CPU oracle.  Prints one JSON line per (net, mode).

    python tools/precision_report.py [--out gpurun_out/precision.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from helpers import synth_sd  # noqa: E402
from s2v_amd import models, ops, synth  # noqa: E402

DEV = "cuda"


def err(a, b):
    a = a.detach().cpu().double().numpy()
    b = np.asarray(b, np.float64)
    d = np.abs(a - b)
    return {"max": float(d.max()), "mean": float(d.mean())}


def clamped(a, b):
    a = a.detach().cpu().double().clamp(0, 1).numpy()
    b = np.clip(np.asarray(b, np.float64), 0, 1)
    d = np.abs(a - b)
    return {"max": float(d.max()), "mean": float(d.mean())}


def probe_err(t, g, name):
    flat = t.detach().cpu().reshape(-1).double().numpy()
    d = np.abs(flat[g[f"{name}_idx"]] - g[f"{name}_val"].astype(np.float64))
    return {"max": float(d.max()), "mean": float(d.mean()), "probe": True}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    G = lambda n: np.load(os.path.join(ROOT, "tests", "golden", f"{n}.npz"))  # noqa: E731
    lnet, enet, dnet = models.LNet(), models.ENet(), models.DNet()
    for m, n in ((lnet, "lnet"), (enet, "enet"), (dnet, "dnet")):
        m.load_state_dict(synth_sd(n))
        m.eval()
    gfp = models.GFPGANv1Clean(out_size=512, num_style_feat=512, channel_multiplier=2, decoder_load_path=None,
                               fix_decoder=False, num_mlp=8, input_is_latent=True, different_w=True, narrow=1,
                               sft_half=True)
    gfp.load_state_dict(synth_sd("gfpgan"))
    gpen = models.FullGenerator(512, 512, 8, 2)
    gpen.load_state_dict(synth_sd("gpen"))
    rows = []
    from oracle import nets
    mel16, face16, gt16 = synth.lipsync_inputs("enet.b16", 16, 256)
    with torch.no_grad():
        ro16, _ = nets.enet_forward(synth_sd("enet"), *(torch.from_numpy(a[:2]) for a in (mel16, face16, gt16)))
    for mode in ("f32", "bf16x3", "f16x3"):
        ops.set_precision(mode)
        g = G("lnet_b2_96")
        mel, face, _ = synth.lipsync_inputs("golden.lnet", 2, 96)
        rows.append({"net": "LNet b2 96", "mode": mode, "out": err(lnet(torch.from_numpy(mel).to(DEV),
                                                                         torch.from_numpy(face).to(DEV)), g["out"])})
        for size in (256, 384):
            g = G(f"enet_b1_{size}")
            mel, face, gt = synth.lipsync_inputs(f"golden.enet{size}", 1, size)
            out, low = enet(*(torch.from_numpy(a).to(DEV) for a in (mel, face, gt)))
            r = {"net": f"ENet b1 {size}", "mode": mode, "low": err(low, g["low"]),
                 "out": err(out, g["out"]) if "out" in g.files else probe_err(out, g, "out")}
            if "out" in g.files:
                r["out_clamped01"] = clamped(out, g["out"])
            rows.append(r)
        out16, _ = enet(*(torch.from_numpy(a).to(DEV) for a in (mel16, face16, gt16)))
        rows.append({"net": "ENet b16 256 (frames 0-1 vs CPU oracle)", "mode": mode, "out": err(out16[:2], ro16),
                     "out_clamped01": clamped(out16[:2], ro16)})
        for size, b in ((128, 2), (256, 1)):
            g = G(f"dnet_b{b}_{size}")
            src, coeff = synth.dnet_inputs(f"golden.dnet{size}", b, size)
            o = dnet(torch.from_numpy(src).to(DEV), torch.from_numpy(coeff).to(DEV))
            r = {"net": f"DNet b{b} {size}", "mode": mode, "flow": err(o["flow_field"], g["flow"])}
            for k in ("warp_image", "fake_image"):
                r[k] = err(o[k], g[k]) if k in g.files else probe_err(o[k], g, k)
            rows.append(r)
        g = G("gfpgan_b1_512")
        x = torch.from_numpy(synth.face_inputs("golden.gfpgan", 1)).to(DEV)
        img, rgbs = gfp(x, return_rgb=True, randomize_noise=False)
        rows.append({"net": "GFPGANv1Clean b1 512", "mode": mode, "out": probe_err(img, g, "out")})
        g = G("gpen_b1_512")
        x = torch.from_numpy(synth.face_inputs("golden.gpen", 1)).to(DEV)
        img, _ = gpen(x)
        rows.append({"net": "GPEN-512 b1", "mode": mode, "out": probe_err(img, g, "out")})
    for r in rows:
        print(json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
