set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/exp/fixed_cost.py > gpurun_out/fixed.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/fixed.log | tail -12
exit $rc
