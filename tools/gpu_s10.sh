O=gpurun_out/s10; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
OUT=$O/prof W=lipsync bash tools/prof_lnet.sh
head -40 $O/prof/timeline.txt
