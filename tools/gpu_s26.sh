# conv_x3_nar at two / three waves per SIMD against the LDS tiles
O=gpurun_out/s26; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "nar" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
S2V_NAR_OCC=3 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "nar" > $O/test3.log 2>&1 || { tail -30 $O/test3.log; exit 1; }
tail -1 $O/test.log $O/test3.log
run() { timeout -k 10 240 python -u tools/conv_micro.py "$@" --prec f16x3 --graph --iters 10 2>&1 | grep -v amdgpu.ids; }
for s in "--n 4 --h 512 --w 512 --cin 128 --cout 64" "--n 4 --h 512 --w 512 --cin 64 --cout 64" "--n 4 --h 256 --w 256 --cin 256 --cout 64"; do
  echo "== $s"; run $s --k 3 --tiles 4,16 || exit 1; echo "occ3"; S2V_NAR_OCC=3 run $s --k 3 --tiles 16 || exit 1
done > $O/sweep.txt
grep -E "==|TFLOP|occ" $O/sweep.txt
