set -o pipefail
mkdir -p gpurun_out/prof
true
true
true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/stats_mouth -o run -- python3 bench.py --workload mouth --steps 5 --warmup 2 --no-cpu-baseline --no-alt > gpurun_out/prof/stats_mouth.log 2>&1 || { tail -5 gpurun_out/prof/stats_mouth.log; exit 1; }
python3 tools/rocprof_summary.py gpurun_out/prof/stats_mouth/run_results.db gpurun_out/prof/stats_mouth.csv
head -25 gpurun_out/prof/stats_mouth.csv
