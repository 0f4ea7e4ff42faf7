# fused FFC tests, then LNet bench A/B (S2V_LNET_FUSED 0 / 1, interleaved), then a kernel-trace profile
O=${O:-gpurun_out/ab_lnet}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ffc_gpu.py -x -q --timeout 120 --timeout-method thread > $O/test_ffc.log 2>&1 || { tail -30 $O/test_ffc.log; exit 1; }
tail -2 $O/test_ffc.log
for f in 0 1 0 1; do S2V_LNET_FUSED=$f timeout -k 10 300 python -u bench.py --workload lnet --steps 30 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b$f.log 2>&1 || exit 1; echo "fused=$f $(grep -h '"value"' $O/b$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
OUT=$O/prof bash tools/prof_lnet.sh > /dev/null 2>&1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/ab_lnet/prof/stats.csv")))
for r in rows[:16]:
    print(f"{r['name'][:70]:70s} {r['calls']:>5s} {float(r['avg_us']):8.2f}")
PY
