#!/bin/bash
# r04 session 11: partial-slice 1x1 buffer path: GPU tests, then the rocprof / stamped-roofline consistency check,
# then LNet / lipsync benches
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s11; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
    tests/test_models_gpu.py tests/test_timed_config_gpu.py tests/test_lanes_gpu.py > $O/tests.log 2>&1 || exit $?
echo tests ok
bash tools/r04_prof_check.sh || exit $?
for w in lnet lipsync lnet lipsync; do
  echo "== $w" >> $O/bench.log
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-alt \
    --no-roofline >> $O/bench.log 2>&1 || exit $?
done
echo done
