#!/bin/bash
# rocprofv3 --pmc passes (each within the per-block counter limits) over the
# tiled GEMM workload; summary -> gpurun_out/pmc_gemm_tile.txt
set -u
cd /tmp; export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
run() { timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmcgt_$2 -o p -- python3 scripts/exp/pmc_gemm_tile.py > gpurun_out/pmcgt_$2.log 2>&1; }
run "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" a || exit $?
run "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" b || exit $?
run "FETCH_SIZE" c || exit $?
python3 scripts/pmc_summary.py $(ls gpurun_out/pmcgt_*/*counter_collection.csv gpurun_out/pmcgt_*/*/*counter_collection.csv 2>/dev/null) > gpurun_out/pmc_gemm_tile.txt 2>&1
cat gpurun_out/pmc_gemm_tile.txt
rm -rf gpurun_out/pmcgt_a gpurun_out/pmcgt_b gpurun_out/pmcgt_c
