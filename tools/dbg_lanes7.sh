#!/bin/bash
# lanes GPU tests on the default path, then tools/dbg_lanes4.py bisecting the old ToRGB composition
OUT=${OUT:-gpurun_out/l7}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_lanes_gpu.py -q --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; case $rc in 124|134|137|139) exit 1;; esac
run() {
  echo "== $*" >> "$OUT/log.txt"
  timeout -k 10 240 env S2V_ENET_OVERLAP=0 S2V_LNET_BRANCHES=0 "$@" python3 -u tools/dbg_lanes4.py >> "$OUT/log.txt" 2>&1
  rc=$?
  case $rc in 0) ;; *) echo "rc=$rc for $*" | tee -a "$OUT/log.txt"; exit 1;; esac
}
run S2V_ENET_FUSED_TORGB=0 S2V_RESIZE_UP2=1
run S2V_ENET_FUSED_TORGB=0 S2V_RESIZE_UP2=0
grep -v amdgpu.ids "$OUT/log.txt" | cut -c1-330
