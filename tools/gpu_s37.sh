# ragged-patch halo: parity; halo vs 512x128 on ENet's 400^2 128-channel shape; benches
O=gpurun_out/s37; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo or nar or test_conv2d" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
run() { timeout -k 10 240 python -u tools/conv_micro.py "$@" --prec f16x3 --graph --iters 10 2>&1 | grep -E "TFLOP"; }
for s in "--n 16 --h 400 --w 400 --cin 128 --cout 128" "--n 16 --h 400 --w 400 --cin 256 --cout 128" "--n 2 --h 360 --w 360 --cin 64 --cout 32" "--n 2 --h 360 --w 360 --cin 160 --cout 32"; do
  echo "== $s"; run $s --k 3 --tiles 0,4,9,18,20 || exit 1
done
