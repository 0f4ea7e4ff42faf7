O=gpurun_out/s09; mkdir -p $O
b() { timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline "$@" > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for r in 1 2; do
for g in half 160 192 0; do echo "lipsync style_grid=$g $(S2V_ENET_STYLE_GRID=$g b --workload lipsync)"; done
done
