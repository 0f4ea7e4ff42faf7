#!/bin/bash
# Interleaved A/B of environment settings on one box (through gpurun, repo root):
#   bash tools/ab_env.sh OUT WORKLOAD REPS "SETTING_A" "SETTING_B" [...]
# e.g. bash tools/ab_env.sh gpurun_out/ab_head dnet 3 "S2V_HEAD_X3=0" "S2V_HEAD_X3=1"
# Each setting is a space-separated list of VAR=value exported for one bench run; the settings run in
# turn REPS times (A B A B ...), each bench under its own time limit; the chain stops at a failure.
set -o pipefail
O=$1; W=$2; REPS=$3; shift 3
mkdir -p "$O"
EXTRA=${EXTRA:---steps 20 --warmup 3}
for rep in $(seq "$REPS"); do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    log="$O/${W}_$i.log"
    ( for kv in $setting; do export "$kv"; done
      timeout -k 10 300 python -u bench.py --workload "$W" $EXTRA --no-cpu-baseline --no-alt --no-roofline > "$log" 2>&1 ) ||
      { echo "FAIL [$setting]"; tail -20 "$log"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(f'rep $rep [{sys.argv[2]}] {d[\"value\"]} {d[\"unit\"]} {d[\"ms_per_step\"]} ms')" "$log" "$setting"
  done
done
