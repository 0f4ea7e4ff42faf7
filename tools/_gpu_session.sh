set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ops_tests.log 2>&1 || { echo OPS_FAIL; tail -30 gpurun_out/ops_tests.log; exit 1; }
tail -2 gpurun_out/ops_tests.log
timeout -k 10 120 python tools/conv_micro.py --n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3 --iters 10 > gpurun_out/micro.log 2>&1 || exit 1
timeout -k 10 120 python tools/conv_micro.py --n 16 --h 200 --w 200 --cin 256 --cout 128 --k 3 --up2 --iters 10 >> gpurun_out/micro.log 2>&1 || exit 1
timeout -k 10 120 python tools/conv_micro.py --n 16 --h 256 --w 256 --cin 256 --cout 256 --k 3 --iters 5 >> gpurun_out/micro.log 2>&1 || exit 1
cat gpurun_out/micro.log
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_enhancers_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/model_tests.log 2>&1 || { echo MODEL_FAIL; grep -E "FAIL|Error|assert" gpurun_out/model_tests.log | head -20; exit 1; }
tail -2 gpurun_out/model_tests.log
timeout -k 10 200 python tools/precision_report.py --out gpurun_out/precision.json > gpurun_out/precision.log 2>&1; cat gpurun_out/precision.log | tail -20
