set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_fused_decode.py > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
(cd ab2 && timeout -k 10 200 python ../scripts/exp/attn_bench.py 2>&1 | grep -v amdgpu.ids | sed 's/^/OLD /')
timeout -k 10 200 python scripts/exp/attn_bench.py 2>&1 | grep -v amdgpu.ids | sed 's/^/NEW /'
