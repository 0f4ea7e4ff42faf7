#!/bin/bash
# r04: LNet's small convs, graph-timed per launch against tile / split-K alternatives, and the fixed
# cost of a dependent launch (tools/kernel_floor.py)
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/tiny}; mkdir -p $O
run() { timeout -k 10 180 "$@" >> $O/conv.log 2>&1 || exit $?; }
timeout -k 10 120 python -u tools/kernel_floor.py > $O/floor.log 2>&1 || exit $?
for shp in "--h 14 --w 14 --cin 1024 --cout 256 --k 3 --pad 0" "--h 14 --w 14 --cin 256 --cout 768 --k 3 --pad 0" \
           "--h 26 --w 26 --cin 256 --cout 64 --k 3 --pad 0" "--h 50 --w 50 --cin 128 --cout 32 --k 3 --pad 0"; do
  echo "== $shp" >> $O/conv.log
  run python -u tools/conv_micro.py --n 16 $shp --prec f16x3 --graph --iters 20 --tiles 0,2,4,5 --splits 0,2,4,6,8,12,16
done
for shp in "--h 1200 --w 1 --cin 96 --cout 96" "--h 12 --w 12 --cin 768 --cout 384" "--h 48 --w 48 --cin 96 --cout 48" \
           "--h 84 --w 1 --cin 768 --cout 768"; do
  echo "== $shp" >> $O/conv.log
  run python -u tools/conv_micro.py --n 16 $shp --k 1 --prec f16x3 --graph --iters 20 --tiles 0,2,4,5,6 --splits 0,2,4
done
