#!/bin/bash
# One GPU session (through gpurun, repo root): GPU tests (up to 10 failures reported), smoke(), then
# the bench items in $BENCH ("workload:arg,arg" items).  Each GPU step has its own time limit; an
# abort / segfault / time limit ends the session there (no further GPU step).
OUT=${OUT:-gpurun_out/chk}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/tests.log" 2>&1
  rc=$?
  tail -1 "$OUT/tests.log"
  grep -E "^FAILED|^ERROR" "$OUT/tests.log" | head -20
  if fatal $rc; then echo "TESTS rc=$rc: stopping"; exit 1; fi
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?
  grep -E "smoke:|Error" "$OUT/smoke.log" | head -5
  if fatal $rc; then echo "SMOKE rc=$rc: stopping"; exit 1; fi
fi
for item in $BENCH; do
  w=${item%%:*}; extra=""; [ "$item" != "$w" ] && extra=${item#*:}; extra=${extra//,/ }
  tag=$(echo "$item" | tr ':, -' '____')
  timeout -k 10 600 python -u bench.py --workload $w $extra > "$OUT/bench_$tag.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "BENCH $item rc=$rc"; tail -5 "$OUT/bench_$tag.log"; fatal $rc && exit 1; continue; fi
  echo "== $item"; tail -1 "$OUT/bench_$tag.log" | cut -c1-1500
done
