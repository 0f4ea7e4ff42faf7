# PMC of conv_x3_halo (tile 18) vs the 128x64 LDS tile on 4x512^2 64 -> 64: VALU / SALU per MFMA, waits, MFMA busy
O=gpurun_out/s44; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
S="--n 4 --h 512 --w 512 --cin 64 --cout 64 --k 3"
for t in 4 18; do
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/t${t}_p$i -o run -- python3 tools/conv_micro.py $S --prec f16x3 --iters 3 --tiles $t > $O/t${t}_p$i.log 2>&1 || { echo "pass $t/$i failed rc=$?"; tail -5 $O/t${t}_p$i.log; exit 1; }
done
python3 tools/pmc_counters.py $(ls -d $O/t${t}_p*/) --match "s2v::conv" --out $O/pmc_t$t.json
done
find $O -name "*counter_collection.csv" -delete
echo done
