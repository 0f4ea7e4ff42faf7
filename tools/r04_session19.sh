#!/bin/bash
# r04 final: FETCH / WRITE PMC passes of dnet / pipeline / enhance (this build), installed as
# profiles/pmc_r04_<w>.json on the box, then the driver-form bench lines of every workload
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/s20}; mkdir -p $O
OUT=$O/prof STATS_WORKLOADS="" PMC_WORKLOADS="${PMC_WL-dnet pipeline enhance}" bash tools/gpu_profile.sh > $O/prof.log 2>&1 || exit $?
for w in ${PMC_WL-dnet pipeline enhance}; do cp $O/prof/pmc_$w.json profiles/pmc_r04_$w.json; done
find $O -name "*.db" -delete
echo "pmc ok"
for w in lipsync lnet dnet pipeline enhance; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 --warmup 5 > $O/bench_$w.log 2>&1 || exit $?
  echo "bench $w ok"
done
