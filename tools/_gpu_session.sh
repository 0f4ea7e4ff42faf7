set -o pipefail
for w in mouth; do
S2V_BENCH_VERBOSE=1 timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline --no-alt > gpurun_out/bench_$w.log 2>&1 || { tail -20 gpurun_out/bench_$w.log; exit 1; }
tail -1 gpurun_out/bench_$w.log | cut -c1-220
grep -E "ms .*launches" gpurun_out/bench_$w.log | head -5
done
