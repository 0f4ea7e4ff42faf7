#!/bin/bash
# rocprofv3 kernel trace of the LNet bench (configs[1]): per-level wall times, one FFC per level
# kernel by kernel, per-kernel stats.  OUT=<dir> (default gpurun_out/proflnet); extra env passes through.
set -o pipefail
OUT=${OUT:-gpurun_out/proflnet}
W=${W:-lnet}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/db" -o run -- \
  python3 bench.py --workload "$W" --steps 5 --warmup 2 --no-cpu-baseline --no-alt --no-roofline > "$OUT/bench.log" 2>&1 || exit $?
db=$(find "$OUT/db" -name run_results.db | head -1)
python3 tools/timeline.py "$db" --lnet > "$OUT/levels.txt" 2>&1
python3 tools/timeline.py "$db" --ffc > "$OUT/ffc.txt" 2>&1
[ "$W" = lipsync ] && python3 tools/timeline.py "$db" > "$OUT/timeline.txt" 2>&1
python3 tools/rocprof_summary.py "$db" "$OUT/stats.csv"
rm -f "$db"
echo "prof $W done"
