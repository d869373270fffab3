set -e
cd /tmp; export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
run() { timeout -s KILL 90 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/pmc_$2 -o p -- python3 scripts/exp/attn_one.py > gpurun_out/pmc_$2.log 2>&1; }
run "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC" a
run "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU" b
