#!/bin/bash
# r04: kernel traces of the enhance and dnet benches (stats by symbol / by grid) and their bench lines
set -o pipefail
OUT=${OUT:-gpurun_out/prof2}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in ${WL:-dnet enhance}; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-alt > "$OUT/bench_$w.log" 2>&1 || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/$w" -o run -- \
    python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-alt --no-roofline > "$OUT/$w.log" 2>&1 || exit $?
  db=$(find "$OUT/$w" -name run_results.db | head -1)
  python3 tools/rocprof_summary.py "$db" "$OUT/stats_$w.csv"
  python3 tools/rocprof_summary.py "$db" "$OUT/stats_${w}_by_grid.csv" --by-grid
  rm -f "$db"
  echo "$w done"
done
