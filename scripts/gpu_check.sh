#!/bin/bash
# GPU-box check: build, GPU tests, bench, optional rocprofv3 kernel profile.
# Every GPU step has its own time limit; a crash-class exit code (abort,
# segfault, timeout) stops the script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

python -m loqa_hub_amd._native.build > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-420} python -m pytest tests -m gpu -x -q -p no:cacheprovider ${TEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -25 gpurun_out/gpu_tests.log
  if crash $rc; then echo "gpu tests crashed rc=$rc - stopping"; exit $rc; fi
fi

if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-420} python bench.py --steps ${STEPS:-3} --warmup ${WARMUP:-1} ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/bench.log | tail -3
  if [ $rc != 0 ]; then echo "bench rc=$rc - stopping"; exit $rc; fi
fi

if [ "${PROFILE:-0}" = 1 ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 ${PROF_TIMEOUT:-420} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 2 --warmup 1 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?
  echo "profile rc=$rc"
  python scripts/kernel_summary.py gpurun_out/prof/run_kernel_stats.csv 30 || true
fi
