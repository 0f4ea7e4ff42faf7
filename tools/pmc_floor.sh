#!/bin/bash
# PMC passes over the 1-block 1-slice conv launch chain of tools/kernel_floor.py (--case $CASE): where the
# fixed per-launch cost of a small split-precision conv goes (instruction fetch, waits, busy cycles).
O=${O:-gpurun_out/pmcfloor}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/kernel_floor.py --n 50 --case ${CASE:-0} > $O/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $O/p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_counters.py $(ls -d $O/p*/) --match "${MATCH:-s2v::}" --out $O/pmc.json
cat $O/pmc.json
