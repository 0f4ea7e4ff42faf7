#!/bin/bash
# Round profiling session on one MI355X (run through gpurun from the repo root):
#   rocprofv3 --kernel-trace --stats of each bench workload (graph replay, as benchmarked), then
#   two PMC passes (FETCH_SIZE, WRITE_SIZE) of the given workloads (eager, one dispatch per op).
# Every GPU step has its own time limit and the chain stops at the first failure.
set -e
set -o pipefail
OUT=${OUT:-gpurun_out/prof}
PMC_WORKLOADS=${PMC_WORKLOADS-lipsync}
STATS_WORKLOADS=${STATS_WORKLOADS-"lipsync lnet pipeline enhance mouth"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in $STATS_WORKLOADS; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$w" -o run -- \
    python3 bench.py --workload "$w" --steps 5 --warmup 2 --no-cpu-baseline --no-alt > "$OUT/stats_$w.log" 2>&1
  python3 tools/rocprof_summary.py "$OUT/stats_$w/run_results.db" "$OUT/stats_$w.csv"
  echo "stats $w done"
done
for w in $PMC_WORKLOADS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 500 rocprofv3 --pmc "$c" --output-format csv -d "$OUT/pmc_${w}_$c" -o run -- \
      python3 bench.py --workload "$w" --no-graph --steps 1 --warmup 1 --no-roofline --no-cpu-baseline --no-alt \
      > "$OUT/pmc_${w}_$c.log" 2>&1
    echo "pmc $w $c done"
  done
  python3 tools/pmc_traffic.py "$OUT/pmc_${w}_FETCH_SIZE" "$OUT/pmc_${w}_WRITE_SIZE" "$OUT/pmc_$w.json" "$w"
  if [ -f "$OUT/stats_$w.csv" ]; then python3 tools/hbm_report.py "$OUT/pmc_$w.json" "$OUT/stats_$w.csv" "$OUT/hbm_$w.json" "$w"; fi
done
