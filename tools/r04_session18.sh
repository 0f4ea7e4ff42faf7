#!/bin/bash
# r04 final bench lines (headline roofline per launch shape) + the rocprof-by-grid check of the lipsync bench
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/s18}; mkdir -p $O
for w in lipsync lnet dnet pipeline enhance; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 > $O/bench_$w.log 2>&1 || exit $?
  echo "bench $w ok"
done
OUT=$O/profcheck bash tools/r04_prof_check.sh || exit $?
