#!/bin/bash
# r04 perf-db: add the enhancer workload's keys to the table, GPU suite with the table, A/B of enhance
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/s15}; mkdir -p $O
cp speech-to-video-mpp_amd/perfdb_mi355x.json $O/perfdb_mi355x.json
timeout -k 10 900 python -u tools/tune_perfdb.py enhance --merge --out $O/perfdb_mi355x.json --raw $O/perfdb_raw_enhance.json \
  > $O/tune.log 2>&1 || exit $?
echo "tune ok"
cp $O/perfdb_mi355x.json speech-to-video-mpp_amd/perfdb_mi355x.json
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || exit $?
echo "tests ok"
bash tools/r04_ab_env.sh $O enhance 2 "S2V_PERFDB=0" "S2V_PERFDB=1" || exit $?
echo "ab enhance ok"
