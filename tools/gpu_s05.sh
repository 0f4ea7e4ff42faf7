O=gpurun_out/s05; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ffc_gpu.py -x -v --timeout 120 --timeout-method thread > $O/test_ffc.log 2>&1; rc=$?
tail -25 $O/test_ffc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_timed_config_gpu.py -x -q --timeout 200 --timeout-method thread -k "lnet or enet or lipsync" > $O/test_models.log 2>&1; rc=$?
tail -5 $O/test_models.log
[ $rc -eq 0 ] || exit $rc
for f in 1 0; do S2V_LNET_FUSED=$f timeout -k 10 300 python -u bench.py --workload lnet --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/bench_lnet_fused$f.log 2>&1 || exit 1; done
grep -h '"value"' $O/bench_lnet_fused*.log | python3 -c "import sys,json; [print(json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
