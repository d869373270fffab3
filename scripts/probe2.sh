set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python scripts/exp/run_gemv_exp.py v2 > gpurun_out/exp1.log 2>&1; rc=$?
tail -3 gpurun_out/exp1.log; exit $rc
