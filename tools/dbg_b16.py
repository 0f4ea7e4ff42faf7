#!/usr/bin/env python3
"""Debug: ENet(+LNet) B=16 vs the CPU oracle on 2 frames, under the env knobs given on the
command line (run one configuration per process)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import s2v_import  # noqa: E402,F401
from helpers import synth_sd  # noqa: E402
from oracle import nets  # noqa: E402
from s2v_amd import models, ops, synth  # noqa: E402

B = int(os.environ.get("DBG_B", "16"))
prec = os.environ.get("DBG_PREC", "f16x3")
ops.set_precision(prec)
m = models.ENet()
sd = synth_sd("enet")
m.load_state_dict(sd)
m.eval()
mel, face, gt = synth.lipsync_inputs("enet.b16", B, 256)
dev = "cuda"
outs = []
for rep in range(2):
    out, low = m(torch.from_numpy(mel).to(dev), torch.from_numpy(face).to(dev), torch.from_numpy(gt).to(dev))
    torch.cuda.synchronize()
    outs.append((out.cpu(), low.cpu()))
with torch.no_grad():
    ro, rl = nets.enet_forward(sd, torch.from_numpy(mel[:2]), torch.from_numpy(face[:2]), torch.from_numpy(gt[:2]))
o, lo = outs[0]
print(f"B={B} {prec} env={ {k: v for k, v in os.environ.items() if k.startswith('S2V_')} }: "
      f"out {float((o[:2] - ro).abs().max()):.3e} low {float((lo[:2] - rl).abs().max()):.3e} "
      f"rep-equal {torch.equal(outs[0][0], outs[1][0])}", flush=True)
