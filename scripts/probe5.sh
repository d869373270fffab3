set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python scripts/bench_configs.py --config 2 3 > gpurun_out/cfg23.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/cfg23.log | tail -4
exit $rc
