#!/bin/bash
# One GPU session through gpurun (repo root): the GPU test suite, smoke(), then the bench
# workloads named in $BENCH ("name:extra args" items).  Each GPU step has its own time limit; the
# chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/chk}
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > "$OUT/tests.log" 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" "$OUT/tests.log" | head -30; tail -5 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  grep smoke: "$OUT/smoke.log"
fi
for item in $BENCH; do
  w=${item%%:*}; extra=""; [ "$item" != "$w" ] && extra=${item#*:}; extra=${extra//,/ }
  timeout -k 10 600 python -u bench.py --workload $w $extra > "$OUT/bench_$w.log" 2>&1 || { echo "BENCH $w FAIL"; tail -20 "$OUT/bench_$w.log"; exit 1; }
  tail -1 "$OUT/bench_$w.log" | cut -c1-2500
done
