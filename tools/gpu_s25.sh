# narrow conv (4x512^2 64->64 3x3): deep-stage tiles, and PMC of the LDS tile vs conv_x3_nar
O=gpurun_out/s25; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
S="--n 4 --h 512 --w 512 --cin 64 --cout 64 --k 3"
timeout -k 10 240 python -u tools/conv_micro.py $S --prec f16x3 --graph --iters 10 --tiles 4,13,14,15,16 2>&1 | grep -E "TFLOP|rror" || exit 1
for t in 4 16; do
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/t${t}_p$i -o run -- python3 tools/conv_micro.py $S --prec f16x3 --iters 3 --tiles $t > $O/t${t}_p$i.log 2>&1 || { echo "pass $t/$i failed rc=$?"; tail -5 $O/t${t}_p$i.log; exit 1; }
done
python3 tools/pmc_counters.py $(ls -d $O/t${t}_p*/) --match "s2v::conv" --out $O/pmc_t$t.json
done
python3 - <<'P'
import json
for t in (4, 16):
    d = json.load(open(f"gpurun_out/s25/pmc_t{t}.json"))
    print(t, json.dumps(d)[:1500])
P
