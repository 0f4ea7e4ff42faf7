#!/bin/bash
# LDS-DMA ring conv tiles (force_tile 13..18) against the planner's choice on LNet's FFC GEMM shapes at
# B = 16 (f16x3, conv_micro), split-K 1 / 2 / 4 / 8.
cd "$GRAFT_REPO_ROOT"
T=${TILES:-0,13,14,15,16,17,18}
S=${SPLITS:-1,2,4,8}
while read -r name args; do
  [ -z "$name" ] && continue
  echo "== $name"
  timeout -k 10 120 python -u tools/conv_micro.py $args --prec f16x3 --iters 20 --graph --tiles $T --splits $S 2>&1 | grep -E "tile=|Error"
  rc=${PIPESTATUS[0]}; case $rc in 124|134|137|139) echo "stop rc=$rc"; exit 1;; esac
done <<'SHAPES'
c2l12 --n 16 --h 14 --w 14 --cin 1024 --cout 256 --k 3 --pad 0
l2g12 --n 16 --h 14 --w 14 --cin 256 --cout 768 --k 3 --pad 0
st1_12 --n 16 --h 12 --w 12 --cin 768 --cout 384 --k 1
fu12 --n 16 --h 84 --w 1 --cin 768 --cout 768 --k 1
st2_12 --n 16 --h 12 --w 12 --cin 384 --cout 768 --k 1
c2l24 --n 16 --h 26 --w 26 --cin 256 --cout 64 --k 3 --pad 0
l2g24 --n 16 --h 26 --w 26 --cin 64 --cout 192 --k 3 --pad 0
st1_24 --n 16 --h 24 --w 24 --cin 192 --cout 96 --k 1
fu24 --n 16 --h 312 --w 1 --cin 192 --cout 192 --k 1
st2_24 --n 16 --h 24 --w 24 --cin 96 --cout 192 --k 1
c2l48 --n 16 --h 50 --w 50 --cin 128 --cout 32 --k 3 --pad 0
l2g48 --n 16 --h 50 --w 50 --cin 32 --cout 96 --k 3 --pad 0
st1_48 --n 16 --h 48 --w 48 --cin 96 --cout 48 --k 1
fu48 --n 16 --h 1200 --w 1 --cin 96 --cout 96 --k 1
SHAPES
