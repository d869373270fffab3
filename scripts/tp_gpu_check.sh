set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_custom_allreduce_gpu.py tests/test_tp_gpu.py -x -v -s --timeout 560 --timeout-method thread -p no:cacheprovider > gpurun_out/tp_tests.log 2>&1
rc=$?
tail -30 gpurun_out/tp_tests.log
exit $rc
