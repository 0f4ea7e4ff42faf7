#!/bin/bash
# per-launch conv timings (serialised pre-pass, S2V_BENCH_VERBOSE=2) of dnet / enhance / lnet
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/s13}; mkdir -p $O
for w in dnet enhance lnet; do
  S2V_BENCH_VERBOSE=2 timeout -k 10 300 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-alt \
    > $O/$w.json 2> $O/$w.verbose || exit $?
  echo "$w ok"
done
