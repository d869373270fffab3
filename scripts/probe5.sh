set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_configs.py --config 3 > gpurun_out/cfg3.log 2>&1 || { tail -5 gpurun_out/cfg3.log; exit 1; }
grep '^{' gpurun_out/cfg3.log
timeout -k 10 800 python scripts/bench_configs.py --config 5 --per-stream 3 > gpurun_out/cfg5.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/cfg5.log | tail -3
exit $rc
