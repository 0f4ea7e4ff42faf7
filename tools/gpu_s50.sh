# GFPGANer restore composition: new GPU tests + the face / enhancer tests whose kernels it touches
O=gpurun_out/${OUT:-s50}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_restore_gpu.py tests/test_face_gpu.py > $O/t.log 2>&1; rc=$?
tail -30 $O/t.log; exit $rc
