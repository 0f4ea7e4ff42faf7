#!/bin/bash
# r04: rocprof of the lipsync bench without the roofline pre-passes (every launch of the dominant symbols is a
# graph replay or one of the few eager calibration / capture forwards), by symbol and by grid, phase timeline;
# then the same bench command's stamped roofline for comparison
set -o pipefail
OUT=${OUT:-gpurun_out/profcheck}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/lipsync" -o run -- \
  python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-alt --no-roofline > "$OUT/lipsync.log" 2>&1 || exit $?
db=$(find "$OUT/lipsync" -name run_results.db | head -1)
python3 tools/rocprof_summary.py "$db" "$OUT/stats_lipsync.csv"
python3 tools/rocprof_summary.py "$db" "$OUT/stats_lipsync_by_grid.csv" --by-grid
python3 tools/timeline.py "$db" --steps 3 > "$OUT/timeline_lipsync.txt"
rm -f "$db"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-alt > "$OUT/bench_stamped.log" 2>&1 || exit $?
echo done
