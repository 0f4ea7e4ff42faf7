# default bench.py contract line on the final tree
O=gpurun_out/${OUT:-s55}; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '"metric"' $O/bench.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"])'
