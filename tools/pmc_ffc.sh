#!/bin/bash
# PMC passes over tools/ffc_micro.py (fused FFC kernels vs the separate launches, B = 16, every level).
O=${O:-gpurun_out/pmcffc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
           "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/ffc_micro.py --iters 3 > $O/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $O/p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_counters.py $(ls -d $O/p*/) --match "${MATCH:-s2v::}" --out $O/pmc.json
