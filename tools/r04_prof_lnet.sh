#!/bin/bash
# rocprofv3 kernel traces of the LNet bench with the grouped FFC launch (S2V_LNET_GROUP=1) and with the
# three side-stream branches (=0): per-level wall times and one FFC per level kernel by kernel.
set -o pipefail
OUT=${OUT:-gpurun_out/proflnet}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in 1 0; do
  S2V_LNET_GROUP=$g timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/g$g" -o run -- \
    python3 bench.py --workload lnet --steps 5 --warmup 2 --no-cpu-baseline --no-alt --no-roofline > "$OUT/g$g.log" 2>&1 || exit $?
  db=$(find "$OUT/g$g" -name run_results.db | head -1)
  python3 tools/timeline.py "$db" --lnet > "$OUT/levels_g$g.txt"
  python3 tools/timeline.py "$db" --ffc > "$OUT/ffc_g$g.txt"
  python3 tools/rocprof_summary.py "$db" "$OUT/stats_g$g.csv"
  rm -f "$db"
  echo "g$g done"
done
