#!/bin/bash
# r04 session 8: halo chunk-per-block + single-image input scale: GPU tests, A/B against ab/ on enhance / dnet /
# lipsync / lnet, per-launch lists
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s8; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
    tests/test_models_gpu.py tests/test_enhancers_gpu.py > $O/tests.log 2>&1 || exit $?
echo tests ok
for w in enhance dnet lipsync lnet; do
  for side in new old new old; do
    root=.; [ $side = old ] && root=ab
    echo "== $side" >> $O/$w.log
    timeout -k 10 300 python -u $root/bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-alt \
      --no-roofline >> $O/$w.log 2>&1 || exit $?
  done
  echo "$w ab ok"
done
for w in dnet enhance; do
  S2V_BENCH_VERBOSE=2 timeout -k 10 300 python -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline \
    --no-alt > $O/launches_$w.log 2>&1 || exit $?
done
echo done
