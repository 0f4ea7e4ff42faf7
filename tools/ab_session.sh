#!/bin/bash
# A/B of two library builds on one box: ./ (new) against ab/ (a copy of the package with the previous
# build's .so files, bench.py and tools/conv_micro.py).  Conv shapes graph-timed, then benches, in
# alternating order.  Usage: bash tools/ab_session.sh OUTDIR [bench workloads ...]
cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/ab}; shift; mkdir -p $O
run() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" >> $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
SHAPES=(
  "--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3"
  "--n 16 --h 128 --w 128 --cin 256 --cout 256 --k 3"
  "--n 16 --h 400 --w 400 --cin 128 --cout 128 --k 3"
  "--n 16 --h 14 --w 14 --cin 1024 --cout 256 --k 3 --pad 0"
  "--n 16 --h 48 --w 48 --cin 256 --cout 256 --k 3"
)
for rep in 1 2; do
  for side in new old; do
    root=.; [ $side = old ] && root=ab
    for s in "${SHAPES[@]}"; do
      echo "== $side $s" >> $O/conv.log
      run conv 120 python -u $root/tools/conv_micro.py $s --prec f16x3 --graph --iters 20
    done
  done
done
for w in "$@"; do
  for side in new old new old; do
    root=.; [ $side = old ] && root=ab
    echo "== $side" >> $O/bench_$w.log
    run bench_$w 300 python -u $root/bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-alt --no-roofline
  done
done
