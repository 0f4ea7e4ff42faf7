#!/bin/bash
# r04 final build check: full GPU suite, bench lines of the workloads (driver command form), rocprof kernel
# stats of lipsync / lnet / dnet / enhance, FETCH_SIZE / WRITE_SIZE passes of lipsync and lnet, PMC of the
# headline conv shape.  Each GPU step has its own limit; the chain stops at the first failure.
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/final}; mkdir -p $O
timeout -k 10 1200 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || exit $?
echo "tests ok"
for w in ${BENCH_WL-lipsync lnet dnet pipeline enhance}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 > $O/bench_$w.log 2>&1 || exit $?
  echo "bench $w ok"
done
OUT=$O/prof STATS_WORKLOADS="${STATS_WL-lipsync lnet dnet enhance}" PMC_WORKLOADS="${PMC_WL-lipsync lnet}" \
  bash tools/gpu_profile.sh > $O/prof.log 2>&1 || exit $?
echo "prof ok"
OUT=$O/pmcconv CONV="--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3 --tiles 1 --prec f16x3 --iters 5" \
  bash tools/pmc_conv.sh > $O/pmcconv.log 2>&1 || exit $?
echo "pmcconv ok"
find $O -name "*.db" -delete
