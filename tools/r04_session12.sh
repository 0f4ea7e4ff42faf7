#!/bin/bash
# r04 in-kernel split-K fold: GPU suite, then interleaved A/B (S2V_SPLITK_FOLD=0 / 1) of the workloads.
cd "$GRAFT_REPO_ROOT"
O=${O:-gpurun_out/s12}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 || exit $?
echo "tests ok"
for w in ${WLS-lnet dnet enhance lipsync}; do
  bash tools/r04_ab_env.sh $O $w 2 "S2V_SPLITK_FOLD=0" "S2V_SPLITK_FOLD=1" || exit $?
  echo "ab $w ok"
done
