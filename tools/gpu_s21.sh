O=gpurun_out/s21; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_enhancers_gpu.py tests/test_timed_config_gpu.py -x -q --timeout 200 --timeout-method thread -k "demod or enhanc or gfpgan or gpen or lipsync_b16" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
b() { timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline --workload $1 > $O/b_$1.log 2>&1 || return 1; grep -h '"value"' $O/b_$1.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
echo "enhance $(b enhance)"
echo "lipsync $(b lipsync)"
echo "enhance $(b enhance)"
echo "lipsync $(b lipsync)"
