# GFPGAN polyphase up-StyleConvs: enhancer / restore / ENet parity, then A/B on the enhance workload
O=gpurun_out/${OUT:-s57}; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_enhancers_gpu.py tests/test_restore_gpu.py tests/test_models_gpu.py > $O/t.log 2>&1 || { grep -E "FAILED|Error|assert" $O/t.log | head -20; tail -5 $O/t.log; exit 1; }
tail -2 $O/t.log
b() { timeout -k 10 300 env $1 python -u bench.py --workload $2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in 1 2 3; do for v in S2V_GFPGAN_POLY_UP=0 S2V_GFPGAN_POLY_UP=1; do r=$(b $v enhance) || exit 1; echo "enhance $v $r"; done; done
