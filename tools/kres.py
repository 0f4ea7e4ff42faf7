#!/usr/bin/env python3
"""Register / scratch / occupancy summary of every kernel in one HIP source compiled for gfx950:
    python tools/kres.py speech-to-video-mpp_amd/csrc/conv_x3.hip [name-regex]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "."
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o",
                      "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\S+) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if re.search(pat, r["name"]):
        g = r.get
        print(f"{g('VGPRs', '?'):>4}v {g('AGPRs', '?'):>4}a scratch {g('ScratchSize', '?'):>4} "
              f"occ {g('Occupancy', '?')} lds {g('LDS Size', '?'):>6}  {r['name']}")
