# A/B: HEAD before conv_cpar_1x1 (ab/) vs the working tree, interleaved on one box
O=gpurun_out/s47; mkdir -p $O
b() { timeout -k 10 300 python -u $1/bench.py --workload $2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in 1 2; do for w in enhance sr; do for r in ab .; do echo "$w $r $(b $r $w)"; done; done; done
