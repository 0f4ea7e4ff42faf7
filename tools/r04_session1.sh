#!/bin/bash
# r04 session 1: tests touched by the ring kernels / grid cap / range guard / timed configuration,
# then the ring and K-scaling sweeps (graph-timed).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py tests/test_range_gpu.py tests/test_timed_config_gpu.py tests/test_torch_ops_gpu.py \
  > gpurun_out/s1/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/s1/tests.log; tail -5 gpurun_out/s1/tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/kscale.sh > gpurun_out/s1/kscale.log 2>&1 || exit 1
bash tools/ring_sweep.sh > gpurun_out/s1/ring_sweep_graph.log 2>&1
