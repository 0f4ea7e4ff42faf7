#!/bin/bash
# PMC passes over one bench workload (eager, one dispatch per op), one rocprofv3 run per pass under its
# own time limit, then the counters of one kernel launch shape (MATCH symbol substring, GRID work-items):
#   WORKLOAD=lipsync MATCH="conv_igemm_x3<256, 256" GRID=2572288 OUT=gpurun_out/pmc bash tools/pmc_workload.sh
# Passes: SQ wave / instruction counters, MFMA-busy / LDS counters, FETCH_SIZE, WRITE_SIZE.
set -e
set -o pipefail
OUT=${OUT:-gpurun_out/pmcw}
W=${WORKLOAD:-lipsync}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_COUNT" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench.py --workload "$W" --no-graph --steps 1 --warmup 1 --no-roofline --no-cpu-baseline --no-alt \
    > "$OUT/p$i.log" 2>&1
  echo "pass $i done"
done
python3 tools/pmc_counters.py $(ls -d $OUT/p*/ ) --match "${MATCH:-conv_igemm}" ${GRID:+--grid $GRID} --out "$OUT/pmc.json"
