set -o pipefail
mkdir -p gpurun_out
run() { echo "== $1"; timeout -k 10 120 python tools/conv_micro.py $1 --iters 20 --prec bf16x3 --tiles $2 2>&1 | grep tile= || exit 1; }
run "--n 16 --h 12 --w 7 --cin 768 --cout 768 --k 1" 0,5,8,9,10
run "--n 16 --h 12 --w 12 --cin 768 --cout 384 --k 1" 0,5,8,9,10
run "--n 16 --h 24 --w 13 --cin 192 --cout 192 --k 1" 0,5,8,9,10
run "--n 16 --h 48 --w 25 --cin 96 --cout 96 --k 1" 0,5,8,9,10
run "--n 16 --h 12 --w 12 --cin 256 --cout 256 --k 3" 0,5,8,9,10
run "--n 16 --h 12 --w 12 --cin 768 --cout 256 --k 3" 0,5,8,9,10
