# A/B: LNet grouped conv pair launched beside the spectral chain (default) vs after its rfft2 (S2V_LNET_PAIR_AFTER_FFT),
# and the 48x48 FFT kernels with their tables in global memory (S2V_FFT48_TG=1)
O=gpurun_out/${OUT:-s49}; mkdir -p $O
S2V_FFT48_TG=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "rfft2" > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in S2V_FFT48_TG=0 S2V_FFT48_TG=1; do echo "== $v" >> $O/micro.log; timeout -k 10 200 env $v python -u tools/ffc_micro.py --iters 20 >> $O/micro.log 2>&1 || exit 1; done
grep -v amdgpu.ids $O/micro.log
b() { timeout -k 10 300 env $1 python -u bench.py --workload $2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in 1 2; do for w in lnet lipsync; do for v in S2V_LNET_PAIR_AFTER_FFT= S2V_LNET_PAIR_AFTER_FFT=48 S2V_LNET_PAIR_AFTER_FFT=12,48 S2V_FFT48_TG=1 S2V_LNET_PAIR_SIDE=1; do r=$(b $v $w) || exit 1; echo "$w $v $r"; done; done; done
