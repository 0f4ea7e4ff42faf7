O=gpurun_out/s06; mkdir -p $O
python3 -c "
import torch, s2v_import
from s2v_amd import ops
p = torch.cuda.get_device_properties(0)
print('arch', p.gcnArchName, 'cus', p.multi_processor_count, 'perfdb', ops.perfdb_applies('cuda:0'), ops.PERFDB_DEVICE)
" > $O/dev.log 2>&1
cat $O/dev.log
for f in 0 1 0 1; do S2V_LNET_FUSED=$f timeout -k 10 300 python -u bench.py --workload lnet --steps 30 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/bench_lnet_fused$f.log 2>&1 || exit 1; echo "fused=$f $(grep -h '"value"' $O/bench_lnet_fused$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
for f in 0 1; do S2V_LNET_FUSED=$f timeout -k 10 300 python -u bench.py --workload lipsync --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/bench_lipsync_fused$f.log 2>&1 || exit 1; echo "lipsync fused=$f $(grep -h '"value"' $O/bench_lipsync_fused$f.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
OUT=$O/prof bash tools/prof_lnet.sh
