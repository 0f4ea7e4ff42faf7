#!/bin/bash
# lipsync / lnet throughput with consecutive steps on 1, 2, 3 lanes (runtime.LaneRunner), interleaved
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/lanes}; mkdir -p $O
for w in lipsync lnet; do
  for rep in 1 2; do
    for l in 1 2 3; do
      echo "== lanes $l" >> $O/$w.log
      timeout -k 10 300 python -u bench.py --workload $w --lanes $l --steps 30 --warmup 6 --no-cpu-baseline --no-alt \
        --no-roofline >> $O/$w.log 2>&1 || exit $?
    done
  done
  echo "$w ok"
done
