# enhance step kernel sequence (rocprofv3 kernel trace, last full step)
O=gpurun_out/${OUT:-s22}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/db -o run -- python3 bench.py --workload enhance --steps 4 --warmup 2 --no-cpu-baseline --no-alt --no-roofline > $O/bench.log 2>&1 || exit 1
db=$(find $O/db -name run_results.db | head -1)
python3 tools/timeline.py "$db" --seq adain_heads2 > $O/seq.txt 2>&1
python3 - "$db" > $O/cols.txt <<'P'
import sqlite3, sys
db = sqlite3.connect(sys.argv[1]); print([r[1] for r in db.execute("pragma table_info(kernels)")])
P
rm -f "$db"
tail -3 $O/seq.txt
