# planner after the ragged-patch / large-N limits: parity of the touched workloads, then benches
O=gpurun_out/s38; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ops_gpu.py tests/test_enhancers_gpu.py tests/test_models_gpu.py tests/test_perfdb_gpu.py tests/test_sr_gpu.py tests/test_timed_config_gpu.py -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
b() { timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline --workload $1 > $O/b_$1.log 2>&1 || return 1; grep -h '"value"' $O/b_$1.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for w in lipsync enhance dnet sr mouth lipsync enhance; do echo "$w $(b $w)"; done
