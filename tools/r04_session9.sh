#!/bin/bash
# r04 session 9: incremental-image epilogue: GPU tests (ops / models / enhancers / pipeline / range / lanes),
# benches of enhance / dnet / lipsync / lnet on this build
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s9; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
    tests/test_models_gpu.py tests/test_enhancers_gpu.py tests/test_pipeline_gpu.py tests/test_range_gpu.py \
    tests/test_lanes_gpu.py tests/test_timed_config_gpu.py > $O/tests.log 2>&1 || exit $?
echo tests ok
for w in enhance dnet lipsync lnet enhance dnet lipsync lnet; do
  echo "== $w" >> $O/bench.log
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-alt \
    --no-roofline >> $O/bench.log 2>&1 || exit $?
done
S2V_BENCH_VERBOSE=2 timeout -k 10 300 python -u bench.py --workload enhance --steps 2 --warmup 1 --no-cpu-baseline \
    --no-alt > $O/launches_enhance.log 2>&1 || exit $?
echo done
