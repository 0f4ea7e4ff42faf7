#!/bin/bash
# tools/dbg_lanes2.py under side-stream variants, each its own process and time limit.
OUT=${OUT:-gpurun_out/lanes2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  timeout -k 10 240 env "$@" python3 -u tools/dbg_lanes2.py >> "$OUT/log.txt" 2>&1
  rc=$?
  case $rc in 0) ;; *) echo "rc=$rc for $*" | tee -a "$OUT/log.txt"; exit 1;; esac
}
run DBG_CASE=both
run DBG_CASE=lanes
run DBG_CASE=peer
run DBG_CASE=lanes S2V_ENET_OVERLAP=0 S2V_LNET_BRANCHES=0
run DBG_CASE=lanes S2V_ENET_OVERLAP=0
run DBG_CASE=lanes S2V_LNET_BRANCHES=0
grep -v " OK" "$OUT/log.txt" | grep -E "\[" | head -60
echo done
