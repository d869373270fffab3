#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "vits" > gpurun_out/r4_g18_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g18_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g18_tests.log | tail -2
