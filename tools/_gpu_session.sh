set -o pipefail
mkdir -p gpurun_out/pmc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; grep -E "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -30; tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
run() { echo "== $1"; timeout -k 10 120 python tools/conv_micro.py $1 --iters 10 --prec bf16x3 --tiles $2 2>&1 | grep tile= || exit 1; }
run "--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3" 1,2
run "--n 16 --h 400 --w 400 --cin 256 --cout 128 --k 3" 2
S2V_BENCH_VERBOSE=1 timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHAPE="--n 16 --h 200 --w 200 --cin 256 --cout 256 --k 3 --iters 3 --prec bf16x3 --tiles 1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 tools/conv_micro.py $SHAPE > gpurun_out/pmc/p1.log 2>&1 || { echo P1_FAIL; tail -5 gpurun_out/pmc/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc/p2 -o run -- python3 tools/conv_micro.py $SHAPE > gpurun_out/pmc/p2.log 2>&1 || { echo P2_FAIL; tail -5 gpurun_out/pmc/p2.log; exit 1; }
