#!/bin/bash
# r04 session 5: GPU suite subset for the up2-polyphase / row-pack / adain2 / prefetched-scale / FFT-XCD build,
# then lnet / dnet / lipsync / enhance benches and an LNet trace with per-FFC dumps
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s5; mkdir -p $O
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" >> $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-alt"
run tests 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
    tests/test_models_gpu.py tests/test_timed_config_gpu.py tests/test_range_gpu.py tests/test_lanes_gpu.py \
    tests/test_pipeline_gpu.py tests/test_enhancers_gpu.py
for w in lnet dnet lipsync enhance; do run bench_$w 300 $B --workload $w; done
S2V_UP2_POLY=0 S2V_ROWPACK=0 run bench_lnet_old 300 $B --workload lnet --no-roofline
S2V_UP2_POLY=0 S2V_ROWPACK=0 run bench_dnet_old 300 $B --workload dnet --no-roofline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/tr" -o run -- python3 bench.py --workload lnet --steps 5 --warmup 2 \
  --no-cpu-baseline --no-alt --no-roofline > "$O/tr.log" 2>&1 || exit $?
db=$(find "$O/tr" -name run_results.db | head -1)
python3 tools/timeline.py "$db" --lnet > "$O/levels.txt"
python3 tools/timeline.py "$db" --ffc > "$O/ffc.txt" 2>&1
python3 tools/rocprof_summary.py "$db" "$O/stats_lnet.csv"
rm -f "$db"
