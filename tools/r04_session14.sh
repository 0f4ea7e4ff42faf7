#!/bin/bash
# r04 perf-db: measure the tuned table (tools/tune_perfdb.py) on this box, install it in the box's copy,
# then interleaved A/B of the workloads with the table off / on.
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/s14}; mkdir -p $O
timeout -k 10 900 python -u tools/tune_perfdb.py lnet dnet lipsync --out $O/perfdb_mi355x.json --raw $O/perfdb_raw.json \
  > $O/tune.log 2>&1 || exit $?
echo "tune ok"
cp $O/perfdb_mi355x.json speech-to-video-mpp_amd/perfdb_mi355x.json
for w in ${WLS-lnet dnet lipsync}; do
  bash tools/r04_ab_env.sh $O $w 2 "S2V_PERFDB=0" "S2V_PERFDB=1" || exit $?
  echo "ab $w ok"
done
