O=gpurun_out/s08; mkdir -p $O
b() { timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline "$@" > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for r in 1 2; do
echo "lnet default(pair,fused24) $(b --workload lnet)"
echo "lnet pair-side $(S2V_LNET_PAIR_SIDE=1 b --workload lnet)"
echo "lnet fused 24,48 $(S2V_LNET_FUSED_LEVELS=24,48 b --workload lnet)"
echo "lnet fused 12,24 $(S2V_LNET_FUSED_LEVELS=12,24 b --workload lnet)"
echo "lnet r04 (no pair, no fused) $(S2V_LNET_PAIR=0 S2V_LNET_FUSED=0 b --workload lnet)"
done
for r in 1 2; do
echo "lipsync default $(b --workload lipsync)"
echo "lipsync r04 $(S2V_LNET_PAIR=0 S2V_LNET_FUSED=0 b --workload lipsync)"
echo "lipsync pair-side $(S2V_LNET_PAIR_SIDE=1 b --workload lipsync)"
done
