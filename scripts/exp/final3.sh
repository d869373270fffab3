# round-end style check (tests, smoke, driver-shaped bench), each step limited
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/final_gpu_tests.log 2>&1 || { tail -30 gpurun_out/final_gpu_tests.log; exit 1; }
tail -2 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/final_bench.log | tail -1 | cut -c1-700
