set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bench_configs.py --config 2 3 > gpurun_out/cfg23b.log 2>&1 || { tail -20 gpurun_out/cfg23b.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cfg23b.log | grep '^{' | cut -c1-700
