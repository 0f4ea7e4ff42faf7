# conv_cpar_1x1: parity (conv cases, enhancers, SR, models, timed configs) and the benches that use it
O=gpurun_out/s46; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_enhancers_gpu.py tests/test_sr_gpu.py tests/test_models_gpu.py tests/test_timed_config_gpu.py tests/test_post_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 python -u tools/plan_syms.py enhance --match cpar > $O/cpar_enhance.txt 2>&1 || exit 1
b() { timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline --workload $1 > $O/b_$1.log 2>&1 || return 1; grep -h '"value"' $O/b_$1.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for w in enhance sr lipsync enhance sr; do echo "$w $(b $w)"; done
