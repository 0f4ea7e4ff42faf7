# A/B: ENet's style-encoder side stream at high priority
O=gpurun_out/${OUT:-s59}; mkdir -p $O
b() { timeout -k 10 300 env $1 python -u bench.py --workload $2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in 1 2; do for v in S2V_STREAM_PRIO_ENET=0 S2V_STREAM_PRIO_ENET=-1; do r=$(b $v lipsync) || exit 1; echo "lipsync $v $r"; done; done
