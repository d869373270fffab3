#!/bin/bash
# Round-end style check on the GPU box (no rebuild: the in-tree .so files are
# what the driver loads): GPU tests, smoke(), bench, rocprofv3 kernel stats +
# decode-step anatomy. Each GPU step has its own limit; any failure stops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final_gpu_tests.log 2>&1 || { tail -30 gpurun_out/final_gpu_tests.log; exit 1; }
tail -2 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1 || { tail -20 gpurun_out/final_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/final_bench.log | tail -1 | cut -c1-400
rm -rf gpurun_out/finalprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/finalprof -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/final_prof.log 2>&1 || { tail -20 gpurun_out/final_prof.log; exit 1; }
f=$(ls gpurun_out/finalprof/run_kernel_trace.csv gpurun_out/finalprof/*/run_kernel_trace.csv 2>/dev/null | head -1)
python scripts/decode_steps.py "$f" llm > gpurun_out/final_anatomy.txt 2>&1
python scripts/decode_steps.py "$f" stt > gpurun_out/final_anatomy_stt.txt 2>&1
head -16 gpurun_out/final_anatomy.txt
rm -f "$f"
