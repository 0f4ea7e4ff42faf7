#!/bin/bash
# tools/dbg_lanes4.py variants, each its own process and time limit.
OUT=${OUT:-gpurun_out/l4b}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  echo "== $*" >> "$OUT/log.txt"
  timeout -k 10 240 env S2V_ENET_OVERLAP=0 S2V_LNET_BRANCHES=0 "$@" python3 -u tools/dbg_lanes4.py >> "$OUT/log.txt" 2>&1
  rc=$?
  case $rc in 0) ;; *) echo "rc=$rc for $*" | tee -a "$OUT/log.txt"; exit 1;; esac
}
run S2V_PRECISION=f16x3
run S2V_RANGE_GUARD=0
run S2V_PRECISION=bf16x3
grep -v amdgpu.ids "$OUT/log.txt"
