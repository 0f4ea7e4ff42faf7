# same-process roofline check: bench (stamps on) under the kernel trace, stamps dumped; then the round's
# profiling: kernel stats of every workload + FETCH/WRITE PMC passes -> profiles/*_r05*
O=gpurun_out/s11; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/st -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-alt --dump-stamps $O/stamps.json > $O/st.log 2>&1 || { tail -5 $O/st.log; exit 1; }
db=$(find $O/st -name run_results.db | head -1)
python3 tools/stamp_vs_trace.py "$db" $O/stamps.json $O/stamp_vs_trace.json > $O/svt.txt 2>&1; cat $O/svt.txt
python3 tools/rocprof_summary.py "$db" $O/st_by_grid.csv --by-grid
rm -f "$db"
OUT=$O/prof STATS_WORKLOADS="lipsync lnet pipeline enhance" PMC_WORKLOADS="lipsync lnet pipeline enhance" bash tools/gpu_profile.sh > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*.db" -delete
find $O/prof -name "*counter_collection.csv" -delete
echo "profile done"
