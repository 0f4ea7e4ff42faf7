# encoder / LNet overlap variants (lipsync, interleaved)
O=gpurun_out/s32; mkdir -p $O
b() { env $1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in 1 2; do for v in S2V_ENET_STYLE_GRID=half S2V_ENET_OVERLAP=0 S2V_ENET_STYLE_GRID=0; do echo "$v $(b $v)"; done; done
