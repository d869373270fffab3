#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_engine_gpu.py -k "hub_server or follower_hang or custom_allreduce" tests/test_tp_gpu.py tests/test_custom_allreduce_gpu.py > gpurun_out/r4_g2_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g2_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r4_g2_tests.log | tail -12
HOLDS="0 25 0 25" bash scripts/exp/r4_hold_ab.sh
