#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for cfg in "DBG_B=2" "DBG_B=16" "DBG_B=16 DBG_PREC=f32" "DBG_B=16 S2V_ENET_OVERLAP=0" "DBG_B=16 S2V_LNET_BRANCHES=0" "DBG_B=16 S2V_ENET_OVERLAP=0 S2V_LNET_BRANCHES=0" "DBG_B=8"; do
  env $cfg timeout -k 10 200 python -u tools/dbg_b16.py 2>&1 | grep -E "B=|Error|error" | tail -3
  rc=${PIPESTATUS[0]}; case $rc in 124|134|137|139) echo "stop rc=$rc"; exit 1;; esac
done
