# narrow-N high-resolution convs of the enhancers (GFPGAN / GPEN 512^2 and 256^2 levels): every x3 tile
O=gpurun_out/s23; mkdir -p $O
run() { timeout -k 10 240 python -u tools/conv_micro.py "$@" --prec f16x3 --graph --iters 10 2>&1 | grep -v amdgpu.ids; }
for s in "--n 4 --h 512 --w 512 --cin 128 --cout 64" "--n 4 --h 512 --w 512 --cin 64 --cout 64" "--n 4 --h 256 --w 256 --cin 256 --cout 128" "--n 4 --h 256 --w 256 --cin 128 --cout 128" "--n 4 --h 512 --w 512 --cin 64 --cout 32"; do
  echo "== $s"; run $s --k 3 --tiles 0,4,5,6,8,10,11,12,16,17,18 || exit 1
done > $O/sweep.txt
cat $O/sweep.txt | grep -E "==|TFLOP" | head -80
