#!/bin/bash
# Interleaved A/B of environment switches on one box: bash tools/r04_ab_env.sh OUT WORKLOAD REPS "ENV_A" "ENV_B" ...
# (each ENV a space-separated list of VAR=value, "-" for none); bench lines appended to OUT/<workload>.log
cd "$GRAFT_REPO_ROOT"
O=$1; W=$2; R=$3; shift 3; mkdir -p $O
for rep in $(seq $R); do
  for envs in "$@"; do
    echo "== $envs" >> $O/$W.log
    [ "$envs" = "-" ] && envs=""
    env $envs timeout -k 10 200 python -u bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-alt \
      --no-roofline >> $O/$W.log 2>&1 || exit $?
  done
done
