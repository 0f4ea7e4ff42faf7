#!/bin/bash
# One parameterised GPU session through gpurun (repo root):
#   TESTS="<pytest args>"   GPU tests (e.g. "tests/test_torch_ops_gpu.py -k half"), optional
#   SMOKE=1                 __graft_entry__.smoke()
#   BENCH="name:args ..."   bench workloads ("lipsync:--no-cpu-baseline,--no-alt"), optional
#   PY="script args"        one python tool run (tools/*.py), optional
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out/run}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $TESTS \
    > "$OUT/tests.log" 2>&1 || { echo TESTS_FAIL; grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -30; tail -5 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  grep smoke: "$OUT/smoke.log"
fi
if [ -n "$PY" ]; then
  timeout -k 10 ${PY_LIMIT:-600} python -u $PY > "$OUT/py.log" 2>&1 || { echo PY_FAIL; tail -30 "$OUT/py.log"; exit 1; }
  tail -${PY_TAIL:-40} "$OUT/py.log"
fi
for item in $BENCH; do
  w=${item%%:*}; extra=""; [ "$item" != "$w" ] && extra=${item#*:}; extra=${extra//,/ }
  timeout -k 10 600 python -u bench.py --workload $w $extra > "$OUT/bench_$w.log" 2>&1 || { echo "BENCH $w FAIL"; tail -20 "$OUT/bench_$w.log"; exit 1; }
  tail -1 "$OUT/bench_$w.log" | cut -c1-${CUT:-1500}
done
