#!/bin/bash
OUT=${OUT:-gpurun_out/up2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  timeout -k 10 120 env "$@" python3 -u tools/dbg_up2.py >> "$OUT/log.txt" 2>&1
  rc=$?
  case $rc in 0) ;; *) echo "rc=$rc for $*" | tee -a "$OUT/log.txt"; tail -3 "$OUT/log.txt"; exit 1;; esac
}
run DBG_MODE=s2v DBG_C=4
run DBG_MODE=s2v DBG_C=256 DBG_H=100
run DBG_MODE=torch DBG_C=4
run DBG_MODE=torch DBG_C=256 DBG_H=100
grep -v amdgpu.ids "$OUT/log.txt" | tail -40
