# A/B: the library at the session start (ab/, 7808d71) vs HEAD, interleaved; then the dnet / enhance bench
# lines with the corrected split-precision peak
O=gpurun_out/s33; mkdir -p $O
b() { timeout -k 10 300 python -u $1/bench.py --workload $2 --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for rep in 1 2; do for w in lnet lipsync enhance; do for r in ab .; do echo "$w $r $(b $r $w)"; done; done; done
for w in dnet enhance; do
  timeout -k 10 420 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_$w.log 2>&1 || { tail -5 $O/bench_$w.log; exit 1; }
  grep -h '^{' $O/bench_$w.log | tail -1 > $O/bench_$w.json
done
