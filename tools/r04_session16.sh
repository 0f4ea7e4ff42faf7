#!/bin/bash
# r04 perf-db with modulated convs: re-tune enhance + lipsync (merge), the perf-db parity test and the GPU
# suite on the new table, then A/B of enhance and lipsync
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/s16}; mkdir -p $O
cp speech-to-video-mpp_amd/perfdb_mi355x.json $O/perfdb_mi355x.json
timeout -k 10 900 python -u tools/tune_perfdb.py enhance lipsync --merge --out $O/perfdb_mi355x.json \
  --raw $O/perfdb_raw.json > $O/tune.log 2>&1 || exit $?
echo "tune ok"
cp $O/perfdb_mi355x.json speech-to-video-mpp_amd/perfdb_mi355x.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || exit $?
echo "tests ok"
for w in enhance lipsync; do
  bash tools/r04_ab_env.sh $O $w 2 "S2V_PERFDB=0" "S2V_PERFDB=1" || exit $?
  echo "ab $w ok"
done
