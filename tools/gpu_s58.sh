# A/B: HIP stream priorities of the side streams (LNet's spectral chain high / ENet's style encoder low)
O=gpurun_out/${OUT:-s58}; mkdir -p $O
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
b() { timeout -k 10 300 env $1 python -u bench.py --workload $2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
V="S2V_STREAM_PRIO_LNET=0 S2V_STREAM_PRIO_LNET=-1 S2V_STREAM_PRIO_ENET=1"
for rep in 1 2; do for v in $V; do r=$(b $v lipsync) || exit 1; echo "lipsync $v $r"; done; done
for v in S2V_STREAM_PRIO_LNET=0 S2V_STREAM_PRIO_LNET=-1; do r=$(b $v lnet) || exit 1; echo "lnet $v $r"; done
