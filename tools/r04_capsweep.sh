#!/bin/bash
# r04: style-encoder grid cap (persistent blocks beside LNet) re-swept on the r04 build, interleaved reps
cd "$GRAFT_REPO_ROOT"
bash tools/r04_ab_env.sh gpurun_out/capsweep lipsync 2 - "S2V_ENET_STYLE_GRID=96" "S2V_ENET_STYLE_GRID=112" \
  "S2V_ENET_STYLE_GRID=144" "S2V_ENET_STYLE_GRID=160" "S2V_ENET_STYLE_GRID=0"
# one-launch InstanceNorm also at 48^2 (2304-pixel planes; default limit 576)
bash tools/r04_ab_env.sh gpurun_out/capsweep lnet 2 - "S2V_IN_FUSED=2304"
# f16x3 against bf16x3 kernels (graph-timed) at the headline and LNet shapes
O=gpurun_out/capsweep
for shp in "--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3" "--n 16 --h 14 --w 14 --cin 1024 --cout 256 --k 3 --pad 0" \
           "--n 16 --h 48 --w 48 --cin 128 --cout 64 --k 3" "--n 16 --h 12 --w 12 --cin 768 --cout 384 --k 1" \
           "--n 16 --h 400 --w 400 --cin 128 --cout 128 --k 3"; do
  echo "== $shp" >> $O/prec.log
  timeout -k 10 180 python -u tools/conv_micro.py $shp --prec split --graph --iters 20 >> $O/prec.log 2>&1 || exit $?
done
