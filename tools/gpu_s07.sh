O=gpurun_out/s07; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_ffc_gpu.py -x -q --timeout 200 --timeout-method thread -k "d2s or polyphase or enet or lnet or ffc" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
b() { timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline "$@" > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
echo "lnet base $(b --workload lnet)"
echo "lnet pair $(S2V_LNET_PAIR=1 b --workload lnet)"
echo "lnet fused24 $(S2V_LNET_FUSED=1 S2V_LNET_FUSED_LEVELS=24 b --workload lnet)"
echo "lnet fused24+pair $(S2V_LNET_PAIR=1 S2V_LNET_FUSED=1 S2V_LNET_FUSED_LEVELS=24 b --workload lnet)"
echo "lnet base $(b --workload lnet)"
echo "lipsync poly4 $(b --workload lipsync)"
echo "lipsync nopoly4 $(S2V_ENET_POLY_UP4=0 b --workload lipsync)"
echo "lipsync poly4 $(b --workload lipsync)"
echo "lipsync nopoly4 $(S2V_ENET_POLY_UP4=0 b --workload lipsync)"
