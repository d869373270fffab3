set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill_gemm2" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pg2_test.log 2>&1
rc=$?; tail -5 gpurun_out/pg2_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/exp/prefill_gemm2_bench.py > gpurun_out/pg2_bench.log 2>&1
rc=$?; cat gpurun_out/pg2_bench.log | grep -v amdgpu.ids | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 280 python -u scripts/exp/tp8_probe.py --world 8 --layers 4 --stall 90 --serve-timeout 200 > gpurun_out/tp8_probe_default.log 2>&1
rc=$?
grep -v "amdgpu.ids\|socket.cpp\|Gloo" gpurun_out/tp8_probe_default.log | tail -40 | cut -c1-400
exit $rc
