# conv_x3_nar ablation: A loads L1-resident (S2V_NAR_ABL=1, wrong results) vs real
O=gpurun_out/s27; mkdir -p $O
run() { timeout -k 10 240 python -u tools/conv_micro.py "$@" --prec f16x3 --graph --iters 10 2>&1 | grep -E "TFLOP"; }
for s in "--n 4 --h 512 --w 512 --cin 128 --cout 64" "--n 4 --h 512 --w 512 --cin 64 --cout 64"; do
  echo "== $s"; run $s --k 3 --tiles 16 || exit 1; echo abl1; S2V_NAR_ABL=1 run $s --k 3 --tiles 16 || exit 1
done
