#!/bin/bash
# tools/dbg_lanes3.py over its cases, each its own process and time limit.
OUT=${OUT:-gpurun_out/lanes3}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  timeout -k 10 240 env "$@" python3 -u tools/dbg_lanes3.py >> "$OUT/log.txt" 2>&1
  rc=$?
  case $rc in 0) ;; *) echo "rc=$rc for $*" | tee -a "$OUT/log.txt"; tail -5 "$OUT/log.txt"; exit 1;; esac
}
run DBG_CASE=conv
run DBG_CASE=modconv
run DBG_CASE=lnet S2V_LNET_BRANCHES=0
run DBG_CASE=lnet
run DBG_CASE=enet S2V_ENET_OVERLAP=0 S2V_LNET_BRANCHES=0
run DBG_CASE=enet S2V_ENET_OVERLAP=0 S2V_LNET_BRANCHES=0 S2V_PRECISION=f32
grep -v " OK" "$OUT/log.txt" | head -60
echo done
