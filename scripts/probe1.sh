set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
timeout -k 10 300 python scripts/bench_kernels.py fused > gpurun_out/kb1.log 2>&1 || { tail -30 gpurun_out/kb1.log; exit 1; }
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -2
