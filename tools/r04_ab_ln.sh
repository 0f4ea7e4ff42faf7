#!/bin/bash
# A/B of the LayerNorm kernels: ./ (new norm.hip) against ab/ (HEAD build), LN micro + dnet / lnet benches
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/abln}; mkdir -p $O
for rep in 1 2; do
  for side in new old; do
    root=.; [ $side = old ] && root=ab
    echo "== $side" >> $O/ln.log
    timeout -k 10 200 python -u $root/tools/ln_micro.py >> $O/ln.log 2>&1 || exit $?
  done
done
echo "ln ok"
for w in dnet lnet; do
  for side in new old new old; do
    root=.; [ $side = old ] && root=ab
    echo "== $side" >> $O/bench_$w.log
    timeout -k 10 300 python -u $root/bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-alt --no-roofline \
      >> $O/bench_$w.log 2>&1 || exit $?
  done
done
echo "bench ok"
