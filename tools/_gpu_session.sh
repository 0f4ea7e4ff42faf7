set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for w in lipsync lnet; do
timeout -k 10 400 python bench.py --workload $w --no-cpu-baseline --no-alt > gpurun_out/bench_$w.log 2>&1 || { tail -20 gpurun_out/bench_$w.log; exit 1; }
tail -1 gpurun_out/bench_$w.log | cut -c1-200
done
