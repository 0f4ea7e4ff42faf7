# r05 final measurements of the current tree: bench lines (driver defaults + each workload), kernel stats,
# FETCH/WRITE PMC and HBM tables, the lipsync phase timeline, the GPEN native ops' bandwidth
O=gpurun_out/${OUT:-s30}; mkdir -p $O
for w in lipsync lnet dnet pipeline enhance; do
  extra=""; [ $w != lipsync ] && extra="--no-cpu-baseline"
  timeout -k 10 420 python -u bench.py --workload $w $extra > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $O/bench_$w.log; exit 1; }
  grep -h '^{' $O/bench_$w.log | tail -1 > $O/bench_$w.json
  python3 -c "import json,sys; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['unit'], d['ms_per_step'], d['roofline'].get('frac'))"
done
timeout -k 10 120 python -u tools/native_ops_bw.py --out $O/native_ops_bw.json > $O/native.log 2>&1 || { tail -5 $O/native.log; exit 1; }
OUT=$O/proflip W=lipsync bash tools/prof_lnet.sh > $O/proflip.log 2>&1 || { tail -5 $O/proflip.log; exit 1; }
OUT=$O/prof STATS_WORKLOADS="lipsync lnet dnet pipeline enhance" PMC_WORKLOADS="lipsync lnet dnet pipeline enhance" bash tools/gpu_profile.sh > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
find $O -name "*.db" -delete
find $O -name "*counter_collection.csv" -delete
echo "final session done"
