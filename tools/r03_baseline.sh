#!/bin/bash
# Round-3 baseline on one MI355X (through gpurun, repo root): GPU tests, PMC passes of the headline
# conv shape and LNet's 12^2 FFC shapes (tools/pmc_conv.sh), rocprof kernel-trace stats of the
# lipsync and lnet workloads.  Every GPU step has its own time limit; the chain stops at the first
# failure.
set -e
set -o pipefail
OUT=${OUT:-gpurun_out/r03base}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/tests.log" 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" "$OUT/tests.log" | head -30; exit 1; }
  tail -1 "$OUT/tests.log"
fi
# headline StyleConv / style-encoder shape on the 256x256 tile, LNet 12^2 conv_to_l (pre-padded
# 14^2 input, 1024 -> 256) and l2g (256 -> 768)
OUT="$OUT/pmc_hd" CONV="--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3 --prec f16x3 --iters 5" bash tools/pmc_conv.sh
OUT="$OUT/pmc_c2l" CONV="--n 16 --h 14 --w 14 --cin 1024 --cout 256 --k 3 --pad 0 --prec f16x3 --iters 20" bash tools/pmc_conv.sh
OUT="$OUT/pmc_l2g" CONV="--n 16 --h 14 --w 14 --cin 256 --cout 768 --k 3 --pad 0 --prec f16x3 --iters 20" bash tools/pmc_conv.sh
for w in ${STATS_WORKLOADS-lipsync lnet}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$w" -o run -- \
    python3 bench.py --workload "$w" --steps 5 --warmup 2 --no-cpu-baseline --no-alt > "$OUT/stats_$w.log" 2>&1
  python3 tools/rocprof_summary.py "$OUT/stats_$w/run_results.db" "$OUT/stats_$w.csv" || true
  tail -1 "$OUT/stats_$w.log" | cut -c1-400
  echo "stats $w done"
done
