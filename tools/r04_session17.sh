#!/bin/bash
# r04 LayerNorm kernels (dense 4-loads-in-flight statistics, LN_EPT applies): norm / model GPU tests, dnet and
# lnet bench lines, rocprof kernel stats of dnet
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/s17}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_ops_gpu.py \
  tests/test_models_gpu.py tests/test_perfdb_gpu.py -k "layernorm or instnorm or dnet or lnet or perfdb" > $O/tests.log 2>&1 || exit $?
echo "tests ok"
for w in dnet lnet; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-alt > $O/bench_$w.log 2>&1 || exit $?
done
echo "bench ok"
OUT=$O/prof STATS_WORKLOADS="dnet" PMC_WORKLOADS="" bash tools/gpu_profile.sh > $O/prof.log 2>&1 || exit $?
echo "prof ok"
find $O -name "*.db" -delete
