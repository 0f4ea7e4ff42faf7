# restore wiring test + per-phase timing of GFPGANer.enhance
O=gpurun_out/${OUT:-s51}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_inference_gpu.py tests/test_restore_gpu.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
timeout -k 10 200 python -u tools/restore_micro.py --h 720 --w 1280 > $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
timeout -k 10 200 python -u tools/restore_micro.py --h 1080 --w 1920 >> $O/micro.log 2>&1 || { tail -20 $O/micro.log; exit 1; }
grep -v amdgpu.ids $O/micro.log
