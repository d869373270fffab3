# norm kernels with the weights requested alongside the row: kernel tests,
# the Whisper / Llama model-level GPU tests, one default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu > gpurun_out/g32_tests.txt 2>&1 || { tail -30 gpurun_out/g32_tests.txt; exit 1; }
tail -2 gpurun_out/g32_tests.txt
timeout -k 10 400 python bench.py > gpurun_out/g32_bench.log 2>&1 || { tail -20 gpurun_out/g32_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g32_bench.log | tail -1 | cut -c1-200
