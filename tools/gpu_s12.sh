O=gpurun_out/s12; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "split_variants or d2s" > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -1 $O/test.log
run() { timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids; }
for side in mix1 mix0 mix1 mix0; do
  root=.; [ $side = mix0 ] && root=ab
  for s in "--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3" "--n 16 --h 400 --w 400 --cin 128 --cout 128 --k 3"; do
    echo "== $side $s $(run python -u $root/tools/conv_micro.py $s --prec split --graph --iters 20 | grep -E 'f16x3|bf16x3' | tr '\n' ' ')"
  done
done
b() { timeout -k 10 300 python -u $1/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-alt --no-roofline --workload lipsync > $O/b.log 2>&1 || return 1; grep -h '"value"' $O/b.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for side in mix1 mix0 mix1 mix0; do root=.; [ $side = mix0 ] && root=ab; echo "lipsync $side $(b $root)"; done
