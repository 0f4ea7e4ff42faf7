#!/bin/bash
# r04 session 6: GPU tests of the halo / narrow-tile / halves build; LNet + lipsync env A/B (up2 polyphase +
# row-pack vs off, two concurrent halves); the narrow-N tile sweep
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s6; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_ops_gpu.py \
    tests/test_models_gpu.py tests/test_timed_config_gpu.py > $O/tests.log 2>&1 || exit $?
echo tests ok
bash tools/r04_ab_env.sh $O lnet 3 - "S2V_UP2_POLY=0 S2V_ROWPACK=0" || exit $?
echo lnet ab ok
bash tools/r04_ab_env.sh $O lipsync 2 - "S2V_LNET_SPEC_MAIN=0" "S2V_UP2_POLY=0 S2V_ROWPACK=0" "S2V_LNET_HALVES=4" || exit $?
echo lipsync ab ok
bash tools/r04_ab_env.sh $O dnet 2 - "S2V_UP2_POLY=0 S2V_ROWPACK=0" || exit $?
echo dnet ab ok
bash tools/r04_nsweep.sh || exit $?
echo nsweep ok
