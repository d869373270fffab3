set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/exp/barrier_cost.py > gpurun_out/cont.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/cont.log | tail -12
exit $rc
