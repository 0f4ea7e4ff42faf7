#!/bin/bash
# Fixed vs per-K-slice cost of the split-precision conv kernels on a small-M GEMM (LNet 12^2, B = 16,
# 1x1, N = 384): graph-timed (no host launch overhead), x3 64x64 (tile 5) and ring 64x64 (tile 13).
cd "$GRAFT_REPO_ROOT"
for cin in 32 96 192 384 768 1536 3072; do
  timeout -k 10 120 python -u tools/conv_micro.py --n 16 --h 12 --w 12 --cin $cin --cout 384 --k 1 --prec f16x3 \
    --iters 50 --graph --tiles 5,13 --splits 1 2>&1 | grep -E "tile=|Error" | sed "s/^/cin=$cin /"
  rc=${PIPESTATUS[0]}; case $rc in 124|134|137|139) echo "stop rc=$rc"; exit 1;; esac
done
for n in 1 4 16 64; do
  timeout -k 10 120 python -u tools/conv_micro.py --n $n --h 12 --w 12 --cin 768 --cout 384 --k 1 --prec f16x3 \
    --iters 50 --graph --tiles 5,13 --splits 1 2>&1 | grep -E "tile=|Error" | sed "s/^/n=$n /"
  rc=${PIPESTATUS[0]}; case $rc in 124|134|137|139) echo "stop rc=$rc"; exit 1;; esac
done
# headline shape: the 256x256 register-staged tile, planner, and the LDS-DMA kernel on a split input
timeout -k 10 120 python -u tools/conv_micro.py --n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3 --prec f16x3 \
  --iters 10 --graph --tiles 0,1 --glds 2>&1 | grep -E "tile=|glds|split_act|Error" | sed "s/^/hd /"
