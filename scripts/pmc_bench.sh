#!/bin/bash
# Hardware counters of every kernel the headline bench dispatches (one short
# bench run per rocprofv3 --pmc pass, each pass within the per-block counter
# limits, no tracing domains): MFMA busy / bf16 rate, LDS bank conflicts, HBM
# fetch. Summary -> gpurun_out/pmc_${TAG:-bench}.txt (scripts/pmc_summary.py).
# PMC_CMD: another program to count (default: one bench step), e.g.
#   PMC_CMD="python3 scripts/exp/vits_prof.py" TAG=vits bash scripts/pmc_bench.sh
set -u
cd /tmp; export TMPDIR=/tmp; cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  echo "pass $2: $1"
  timeout -s KILL 280 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmcb_$2 -o p -- \
    ${PMC_CMD:-python3 bench.py --steps 1 --warmup 0} > gpurun_out/pmcb_$2.log 2>&1
}
run "SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" a || exit $?
run "FETCH_SIZE GRBM_GUI_ACTIVE" b || exit $?
python3 scripts/pmc_summary.py $(ls gpurun_out/pmcb_*/*counter_collection.csv gpurun_out/pmcb_*/*/*counter_collection.csv 2>/dev/null) > gpurun_out/pmc_${TAG:-bench}.txt 2>&1
head -60 gpurun_out/pmc_${TAG:-bench}.txt
rm -rf gpurun_out/pmcb_a gpurun_out/pmcb_b
