# batched-load RoPE + KV append: kernel tests, LLM engine GPU tests, two benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_mixed_attention.py tests/test_tp_gpu.py -m gpu > gpurun_out/g33_tests.txt 2>&1 || { tail -30 gpurun_out/g33_tests.txt; exit 1; }
tail -2 gpurun_out/g33_tests.txt
for i in 1 2; do
timeout -k 10 400 python bench.py > gpurun_out/g33_bench$i.log 2>&1 || { tail -20 gpurun_out/g33_bench$i.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g33_bench$i.log | tail -1 | cut -c1-160
done
