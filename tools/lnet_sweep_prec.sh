#!/bin/bash
# LNet FFC GEMM shapes at B = 16: planner's kernel in f16x3 against exact f32 (conv_micro), each
# measured twice (the first measurement of a shape runs on a cold clock).
cd "$GRAFT_REPO_ROOT"
while read -r name args; do
  [ -z "$name" ] && continue
  echo "== $name"
  for p in f16x3 f32 f16x3 f32; do
    timeout -k 10 120 python -u tools/conv_micro.py $args --prec $p --iters 40 --tiles 0 2>&1 | grep -E "tile=|Error" | sed "s/^/$p /"
    rc=${PIPESTATUS[0]}; case $rc in 124|134|137|139) echo "stop rc=$rc"; exit 1;; esac
  done
done <<'SHAPES'
c2l12 --n 16 --h 14 --w 14 --cin 1024 --cout 256 --k 3 --pad 0
l2g12 --n 16 --h 14 --w 14 --cin 256 --cout 768 --k 3 --pad 0
st1_12 --n 16 --h 12 --w 12 --cin 768 --cout 384 --k 1
fu12 --n 16 --h 84 --w 1 --cin 768 --cout 768 --k 1
st2_12 --n 16 --h 12 --w 12 --cin 384 --cout 768 --k 1
c2l24 --n 16 --h 26 --w 26 --cin 256 --cout 64 --k 3 --pad 0
l2g24 --n 16 --h 26 --w 26 --cin 64 --cout 192 --k 3 --pad 0
st1_24 --n 16 --h 24 --w 24 --cin 192 --cout 96 --k 1
c2l48 --n 16 --h 50 --w 50 --cin 128 --cout 32 --k 3 --pad 0
l2g48 --n 16 --h 50 --w 50 --cin 32 --cout 96 --k 3 --pad 0
SHAPES
