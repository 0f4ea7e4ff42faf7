#!/bin/bash
# A/B of library builds on one box: the workloads in $WL with the default libs2v.so, then with each
# in-tree variant libs2v_<v>.so ($VARIANTS) copied over it (the box's copy of the tree only).
# The style encoder's grid cap is off (a variant without the persistent form would ignore it).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=speech-to-video-mpp_amd
cp $P/libs2v.so /tmp/libs2v_cur.so
for v in cur $VARIANTS; do
  if [ "$v" = cur ]; then cp /tmp/libs2v_cur.so $P/libs2v.so; else cp $P/libs2v_$v.so $P/libs2v.so; fi
  for w in $WL; do
    timeout -k 10 300 env S2V_ENET_STYLE_GRID=0 python3 -u bench.py --workload $w --no-cpu-baseline --no-alt \
      > gpurun_out/ablib_${v}_$w.log 2>&1
    rc=$?
    r=$(tail -1 gpurun_out/ablib_${v}_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("roofline",{}).get("isolated",{}).get("frac"))' 2>/dev/null)
    echo "$v $w: $r (rc=$rc)"
    case $rc in 124|134|137|139) exit 1;; esac
  done
done
