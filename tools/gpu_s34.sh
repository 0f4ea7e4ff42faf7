# re-tune LNet's perf-db keys with the deep-stage tiles (13-15) among the candidates, then A/B the tables
O=gpurun_out/s34; mkdir -p $O
cp speech-to-video-mpp_amd/perfdb_mi355x.json $O/perfdb_before.json
timeout -k 10 900 python -u tools/tune_perfdb.py lnet --merge --tiles 1,2,3,4,5,6,7,8,9,10,11,12,13,14,15 --raw $O/raw_lnet.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -2 $O/tune.log
cp speech-to-video-mpp_amd/perfdb_mi355x.json $O/perfdb_after.json
b() { S2V_PERFDB_PATH=$O/$1 timeout -k 10 300 python -u bench.py --workload $2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in 1 2; do for w in lnet lipsync; do for t in perfdb_before.json perfdb_after.json; do echo "$w $t $(b $t $w)"; done; done; done
