#!/bin/bash
# bench A/B over environment settings: each item "workload|ENV=V ENV2=V2" on its own process
OUT=${OUT:-gpurun_out/ab}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
while IFS= read -r item; do
  [ -z "$item" ] && continue
  i=$((i+1))
  w=${item%%|*}; envs=${item#*|}; [ "$envs" = "$item" ] && envs=""
  timeout -k 10 300 env $envs python3 -u bench.py --workload $w --no-cpu-baseline --no-alt ${EXTRA} > "$OUT/ab_$i.log" 2>&1
  rc=$?
  v=$(tail -1 "$OUT/ab_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)
  echo "$w [$envs]: $v (rc=$rc)"
  case $rc in 124|134|137|139) exit 1;; esac
done <<< "$AB"
