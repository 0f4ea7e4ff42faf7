# rocprofv3 kernel trace + HBM PMC passes of GFPGANer.enhance's composition at 1920x1080 (tools/restore_micro.py)
set -e
set -o pipefail
OUT=gpurun_out/${OUT:-s61}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_restore" -o run -- \
  python3 tools/restore_micro.py --h 1080 --w 1920 --iters 10 --no-detect > "$OUT/stats_restore.log" 2>&1
python3 tools/rocprof_summary.py "$OUT/stats_restore/run_results.db" "$OUT/stats_restore.csv"
echo "stats done"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc "$c" --output-format csv -d "$OUT/pmc_restore_$c" -o run -- \
    python3 tools/restore_micro.py --h 1080 --w 1920 --iters 3 --no-detect > "$OUT/pmc_restore_$c.log" 2>&1
  echo "pmc $c done"
done
python3 tools/pmc_traffic.py "$OUT/pmc_restore_FETCH_SIZE" "$OUT/pmc_restore_WRITE_SIZE" "$OUT/pmc_restore.json" restore
python3 tools/hbm_report.py "$OUT/pmc_restore.json" "$OUT/stats_restore.csv" "$OUT/hbm_restore.json" restore
grep -v amdgpu.ids "$OUT/stats_restore.log" | tail -8
