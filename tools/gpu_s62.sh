# windowed restore paste: restore / inference tests, then the profile pass of tools/gpu_s61.sh
O=gpurun_out/${OUT:-s62}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_restore_gpu.py tests/test_inference_gpu.py > $O/t.log 2>&1 || { grep -E "FAILED|Error|assert" $O/t.log | head -20; tail -5 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python -u tools/restore_micro.py --h 1080 --w 1920 --no-detect > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
timeout -k 10 200 python -u tools/restore_micro.py --h 720 --w 1280 --no-detect >> $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
grep -v amdgpu.ids $O/micro.log
OUT=${OUT:-s62}_prof bash tools/gpu_s61.sh
