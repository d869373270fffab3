set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python scripts/bench_configs.py --config 5 --per-stream 2 > gpurun_out/cfg5b.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/cfg5b.log | tail -3 | cut -c1-2500
exit $rc
