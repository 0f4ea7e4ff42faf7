#!/bin/bash
# r04 session 3: GPU tests of the grouped-launch build; LNet grouped / branched FFC x encoder branches on /
# off; lipsync; launch floor; lane-graph edge check.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s3; mkdir -p $O
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt"
run tests 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
    tests/test_models_gpu.py tests/test_range_gpu.py tests/test_timed_config_gpu.py
run lnet_g1b1 200 $B --workload lnet
S2V_LNET_BRANCHES=0 run lnet_g1b0 200 $B --workload lnet --no-roofline
S2V_LNET_GROUP=0 run lnet_g0b1 200 $B --workload lnet --no-roofline
S2V_LNET_GROUP=0 S2V_LNET_BRANCHES=0 run lnet_g0b0 200 $B --workload lnet --no-roofline
run lnet_g1b1_again 200 $B --workload lnet --no-roofline
run lipsync 300 $B
S2V_LNET_GROUP=0 run lipsync_g0 300 $B --no-roofline
run floor 120 python -u tools/kernel_floor.py
run graph 300 python -u tools/lane_graph_dot.py --out $O/graph
