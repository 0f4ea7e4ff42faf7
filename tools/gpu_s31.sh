# style-encoder grid cap sweep (lipsync, interleaved), then the r05 phase timeline with the fixed encoder-end marker
O=gpurun_out/s31; mkdir -p $O
b() { S2V_ENET_STYLE_GRID=$1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in 1 2; do for g in 96 112 half 144 160 192; do echo "grid $g $(b $g)"; done; done
OUT=$O/proflip W=lipsync bash tools/prof_lnet.sh > $O/proflip.log 2>&1 || { tail -5 $O/proflip.log; exit 1; }
grep -E "step|wall|ends" $O/proflip/timeline.txt | head -8
