#!/bin/bash
# A/B of the row-strip 4x4 blur: enhancer GPU tests, then enhance bench new (./) vs old (ab/), interleaved
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/abfir}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_enhancers_gpu.py \
  tests/test_perfdb_gpu.py > $O/tests.log 2>&1 || exit $?
echo "tests ok"
for side in new old new old; do
  root=.; [ $side = old ] && root=ab
  echo "== $side" >> $O/bench_enhance.log
  timeout -k 10 300 python -u $root/bench.py --workload enhance --steps 20 --warmup 3 --no-cpu-baseline --no-alt --no-roofline \
    >> $O/bench_enhance.log 2>&1 || exit $?
done
echo "bench ok"
