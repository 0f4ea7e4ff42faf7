#!/bin/bash
# r04: kernel trace of the lipsync bench (stats by symbol and by grid, phase timeline) + the LNet per-FFC dumps
set -o pipefail
OUT=gpurun_out/prof1
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/lipsync" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-alt > "$OUT/lipsync.log" 2>&1 || exit $?
db=$(find "$OUT/lipsync" -name run_results.db | head -1)
python3 tools/rocprof_summary.py "$db" "$OUT/stats_lipsync.csv"
python3 tools/rocprof_summary.py "$db" "$OUT/stats_lipsync_by_grid.csv" --by-grid
python3 tools/timeline.py "$db" --steps 2 > "$OUT/timeline_lipsync.txt"
rm -f "$db"
echo "lipsync done"
OUT=gpurun_out/prof1 bash tools/r04_prof_lnet.sh
