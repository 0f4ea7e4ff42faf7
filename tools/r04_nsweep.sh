#!/bin/bash
# r04: narrow-N split-precision conv tiles against the planner's choice (enhancer / DNet / LNet 64- and
# 32-channel 3x3 layers), graph-timed; plus L2 hit / memory-side read counters of two shapes
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/nsweep; mkdir -p $O
run() { timeout -k 10 180 "$@" >> $O/conv.log 2>&1 || exit $?; }
for shp in "--n 4 --h 512 --w 512 --cin 128 --cout 64" "--n 4 --h 512 --w 512 --cin 64 --cout 64" \
           "--n 16 --h 256 --w 256 --cin 64 --cout 64" "--n 16 --h 256 --w 256 --cin 128 --cout 64" \
           "--n 16 --h 96 --w 96 --cin 64 --cout 64" "--n 16 --h 48 --w 48 --cin 128 --cout 64"; do
  echo "== $shp" >> $O/conv.log
  run python -u tools/conv_micro.py $shp --k 3 --prec f16x3 --graph --iters 10 --tiles 0,8,10,11
done
for shp in "--n 4 --h 512 --w 512 --cin 64 --cout 32" "--n 16 --h 96 --w 96 --cin 32 --cout 32" \
           "--n 4 --h 512 --w 512 --cin 128 --cout 256"; do
  echo "== $shp" >> $O/conv.log
  run python -u tools/conv_micro.py $shp --k 3 --prec f16x3 --graph --iters 10 --tiles 0,6,12
done
for t in 8 10; do
  OUT=$O/pmc$t CONV="--n 4 --h 512 --w 512 --cin 128 --cout 64 --k 3 --tiles $t --prec f16x3 --iters 5" \
    bash tools/pmc_conv.sh > $O/pmc$t.log 2>&1 || exit $?
done
