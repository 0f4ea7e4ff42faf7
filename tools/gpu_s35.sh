# conv_x3_halo with 128 output channels per block (tile 20) vs 64 (18) and the implicit-GEMM tiles on wider layers
O=gpurun_out/s35; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run() { timeout -k 10 240 python -u tools/conv_micro.py "$@" --prec f16x3 --graph --iters 10 2>&1 | grep -E "TFLOP"; }
for s in "--n 4 --h 256 --w 256 --cin 128 --cout 128" "--n 4 --h 512 --w 512 --cin 128 --cout 64" "--n 16 --h 128 --w 128 --cin 256 --cout 256" "--n 16 --h 256 --w 256 --cin 256 --cout 256" "--n 16 --h 128 --w 128 --cin 256 --cout 512" "--n 4 --h 256 --w 256 --cin 256 --cout 256"; do
  echo "== $s"; run $s --k 3 --tiles 0,1,18,20 || exit 1
done
