#!/bin/bash
# Round check on the GPU box: GPU tests, smoke, default bench. Each step has its
# own limit; a failure stops the script before further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --timeout 560 --timeout-method thread -p no:cacheprovider ${TEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -8 gpurun_out/gpu_tests.log
  [ $rc = 0 ] || { echo "gpu tests rc=$rc - stopping"; exit $rc; }
fi
if [ "${SKIP_SMOKE:-0}" != 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/smoke.log | tail -3
  [ $rc = 0 ] || { echo "smoke rc=$rc - stopping"; exit $rc; }
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/bench.log | tail -3 | cut -c1-1500
  [ $rc = 0 ] || { echo "bench rc=$rc - stopping"; exit $rc; }
fi
