#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench workloads + the lipsync phase timeline
set -e
set -o pipefail
OUT=${OUT:-gpurun_out/r03prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in ${STATS_WORKLOADS-lipsync lnet}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$w" -o run -- \
    python3 bench.py --workload "$w" --steps 5 --warmup 2 --no-cpu-baseline --no-alt > "$OUT/stats_$w.log" 2>&1
  db=$(find "$OUT/stats_$w" -name run_results.db | head -1)
  python3 tools/rocprof_summary.py "$db" "$OUT/stats_$w.csv"
  python3 tools/rocprof_summary.py "$db" "$OUT/stats_${w}_by_grid.csv" --by-grid
  if [ "$w" = lipsync ]; then python3 tools/timeline.py "$db" --steps 2 > "$OUT/timeline_$w.txt"; fi
  if [ "$w" = lnet ]; then python3 tools/timeline.py "$db" --lnet > "$OUT/timeline_$w.txt"; fi
  tail -1 "$OUT/stats_$w.log" | cut -c1-300
  echo "stats $w done"
done
