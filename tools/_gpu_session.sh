set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
run() { echo "== $1"; timeout -k 10 120 python tools/conv_micro.py $1 --iters 10 --prec bf16x3 --tiles $2 2>&1 | grep tile= || exit 1; }
run "--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3" 1


S2V_BENCH_VERBOSE=1 timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log
