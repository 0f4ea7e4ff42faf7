#!/bin/bash
# r04 session 10: f16 split without v_fma_mix (X3_F16_MIX=0) against ab/ (v_fma_mix): kernel rates and benches
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_ops_gpu.py -k "conv" \
  > $O/tests.log 2>&1 || exit $?
for side in new old new old; do
  root=.; [ $side = old ] && root=ab
  for shp in "--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3" "--n 16 --h 400 --w 400 --cin 128 --cout 128 --k 3" \
             "--n 4 --h 512 --w 512 --cin 128 --cout 64 --k 3"; do
    echo "== $side $shp" >> $O/conv.log
    timeout -k 10 180 python -u $root/tools/conv_micro.py $shp --prec f16x3 --graph --iters 20 >> $O/conv.log 2>&1 || exit $?
  done
done
for w in lipsync lnet; do
  for side in new old new old; do
    root=.; [ $side = old ] && root=ab
    echo "== $side" >> $O/$w.log
    timeout -k 10 300 python -u $root/bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-alt \
      --no-roofline >> $O/$w.log 2>&1 || exit $?
  done
done
echo done
