# conv_x3_nar: parity (bit-identical to the LDS tile, conv cases) then timing against the LDS tiles
O=gpurun_out/${OUT:-s24}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "nar or halo or test_conv2d" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
run() { timeout -k 10 240 python -u tools/conv_micro.py "$@" --prec f16x3 --graph --iters 10 2>&1 | grep -v amdgpu.ids; }
for s in "--n 4 --h 512 --w 512 --cin 128 --cout 64" "--n 4 --h 512 --w 512 --cin 64 --cout 64" "--n 4 --h 256 --w 256 --cin 128 --cout 128" "--n 4 --h 512 --w 512 --cin 64 --cout 32" "--n 16 --h 256 --w 256 --cin 64 --cout 64" "--n 4 --h 256 --w 256 --cin 256 --cout 64"; do
  echo "== $s"; run $s --k 3 --tiles 4,18,19 || exit 1
done > $O/sweep.txt
grep -E "==|TFLOP" $O/sweep.txt
