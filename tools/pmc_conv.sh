#!/bin/bash
# PMC passes over one conv shape (tools/conv_micro.py), one rocprofv3 run per pass, each under its
# own time limit.  CONV="--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3 --tiles 1 --prec f16x3"
set -e
set -o pipefail
OUT=${OUT:-gpurun_out/pmcconv}
CONV=${CONV:-"--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3 --tiles 1 --prec f16x3 --iters 5"}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python3 tools/conv_micro.py $CONV > "$OUT/time.log" 2>&1
grep -E "tile|glds" "$OUT/time.log"
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_COUNT" $PMC_EXTRA; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- python3 tools/conv_micro.py $CONV > "$OUT/p$i.log" 2>&1
  echo "pass $i done"
done
python3 tools/pmc_counters.py $(ls -d $OUT/p*/ ) --match "${MATCH:-conv_igemm}" --out "$OUT/pmc.json"
