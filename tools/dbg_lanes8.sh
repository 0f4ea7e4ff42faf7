#!/bin/bash
# resize / torgb kernel tests, then tools/dbg_lanes4.py: old ToRGB with the rewritten up2 kernel
# (no side streams), and the default path with side streams
OUT=${OUT:-gpurun_out/l8}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -q -x --timeout 120 --timeout-method thread -k "torgb or up2 or resize" > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; case $rc in 124|134|137|139) exit 1;; esac
run() {
  echo "== $*" >> "$OUT/log.txt"
  timeout -k 10 240 env "$@" python3 -u tools/dbg_lanes4.py >> "$OUT/log.txt" 2>&1
  rc=$?
  case $rc in 0) ;; *) echo "rc=$rc for $*" | tee -a "$OUT/log.txt"; exit 1;; esac
}
run S2V_ENET_OVERLAP=0 S2V_LNET_BRANCHES=0 S2V_ENET_FUSED_TORGB=0
run S2V_ENET_OVERLAP=1 S2V_LNET_BRANCHES=1
run S2V_ENET_OVERLAP=1 S2V_LNET_BRANCHES=0
run S2V_ENET_OVERLAP=0 S2V_LNET_BRANCHES=1
grep -v amdgpu.ids "$OUT/log.txt" | cut -c1-330
