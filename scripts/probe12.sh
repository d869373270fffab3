set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmcA gpurun_out/pmcB
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA -o run -- python scripts/exp/pmc_kernels.py > gpurun_out/pmcA.log 2>&1 || { tail -20 gpurun_out/pmcA.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcB -o run -- python scripts/exp/pmc_kernels.py > gpurun_out/pmcB.log 2>&1 || { tail -20 gpurun_out/pmcB.log; exit 1; }
ls gpurun_out/pmcA gpurun_out/pmcB
python scripts/pmc_summary.py $(ls gpurun_out/pmcA/*counter_collection.csv gpurun_out/pmcA/*/*counter_collection.csv 2>/dev/null | head -1) $(ls gpurun_out/pmcB/*counter_collection.csv gpurun_out/pmcB/*/*counter_collection.csv 2>/dev/null | head -1) | tee gpurun_out/pmc_summary.txt
