#!/bin/bash
# r04 session 4: adain_heads2 + LNet/model tests; LNet and lipsync grouped / branched FFC A/B (3 interleaved
# pairs each); then the dnet / enhance profiles (tools/r04_prof2.sh)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s4; mkdir -p $O
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" >> $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt --no-roofline"
run tests 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ops_gpu.py -k "adain" \
    tests/test_models_gpu.py tests/test_timed_config_gpu.py
for rep in 1 2 3; do
  for g in 1 0; do
    echo "== g$g" >> $O/lnet.log; S2V_LNET_GROUP=$g run lnet 200 $B --workload lnet
    echo "== g$g" >> $O/lipsync.log; S2V_LNET_GROUP=$g run lipsync 200 $B
  done
done
OUT=$O bash tools/r04_prof2.sh
