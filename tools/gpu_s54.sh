# A/B: split-K of the FourierUnit 1x1 convs (st1 / fu / st2) at the 12^2 level vs all levels
O=gpurun_out/${OUT:-s54}; mkdir -p $O
b() { timeout -k 10 300 env $1 python -u bench.py --workload $2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
V="S2V_LNET_SPEC_SPLITS_12=1 S2V_LNET_SPEC_SPLITS_12=2 S2V_LNET_SPEC_SPLITS_12=4 S2V_LNET_SPEC_SPLITS_12=0 S2V_LNET_SPEC_SPLITS=0"
for rep in 1 2; do for v in $V; do r=$(b $v lnet) || exit 1; echo "lnet $v $r"; done; done
for v in $V; do r=$(b $v lipsync) || exit 1; echo "lipsync $v $r"; done
