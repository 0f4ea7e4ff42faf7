#!/bin/bash
# r04 session 2: baseline benches of this build (lipsync / lnet), LNet with serialised FFC branches,
# the per-launch conv list of LNet (isolated, un-graphed), the lane-graph edge check.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s2; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
run lipsync python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt
run lnet python -u bench.py --workload lnet --steps 20 --warmup 3 --no-cpu-baseline --no-alt
S2V_LNET_BRANCHES=0 run lnet_serial python -u bench.py --workload lnet --steps 20 --warmup 3 --no-cpu-baseline --no-alt --no-roofline
S2V_BENCH_VERBOSE=2 run lnet_launches python -u bench.py --workload lnet --steps 2 --warmup 1 --no-cpu-baseline --no-alt
run graph python -u tools/lane_graph_dot.py --out $O/graph
