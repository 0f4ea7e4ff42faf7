set -o pipefail
for w in lnet; do
S2V_BENCH_VERBOSE=1 timeout -k 10 400 python bench.py --workload $w > gpurun_out/bench_$w.log 2>&1 || { tail -20 gpurun_out/bench_$w.log; exit 1; }
tail -1 gpurun_out/bench_$w.log
grep -E "ms .*launches" gpurun_out/bench_$w.log | head -6
done
