#!/bin/bash
# Hardware counters of the four Llama-3-8B decode GEMMs run alone on cold
# weights (scripts/pmc_gemm.py), three rocprofv3 --pmc passes within the
# per-block limits (SQ: MFMA / LDS; TCC: FETCH_SIZE; TCC: the EA read-request
# count itself), reduced with the algorithmic bytes beside the counter bytes
# -> gpurun_out/pmc_gemm.txt.
set -u
cd /tmp; export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# the serving tuner's picks for these shapes (BENCH_r05 fused_gemm_tuning):
# every pass counts the same layouts, and no tuning dispatch is counted
export LOQA_FSPLIT_OVERRIDE="${LOQA_FSPLIT_OVERRIDE:-rope:6144x4096:M16=1,2,1;silu:28672x4096:M16=1,2,4;resid:4096x4096:M16=1,1,1;resid:4096x14336:M16=2,2,1}"
run() {
  echo "pass $2: $1"
  timeout -s KILL 240 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmcg_$2 -o p -- \
    python3 scripts/pmc_gemm.py --shapes gpurun_out/pmc_gemm_shapes_$2.json > gpurun_out/pmcg_$2.log 2>&1
}
run "SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" a || exit $?
run "FETCH_SIZE GRBM_GUI_ACTIVE" b || exit $?
run "TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE" c || { echo "rdreq pass failed (counter name?)"; tail -5 gpurun_out/pmcg_c.log; }
python3 scripts/pmc_summary.py --shapes gpurun_out/pmc_gemm_shapes_a.json \
  $(ls gpurun_out/pmcg_*/*counter_collection.csv gpurun_out/pmcg_*/*/*counter_collection.csv 2>/dev/null) \
  > gpurun_out/pmc_gemm.txt 2>&1
head -40 gpurun_out/pmc_gemm.txt
rm -rf gpurun_out/pmcg_a gpurun_out/pmcg_b gpurun_out/pmcg_c
