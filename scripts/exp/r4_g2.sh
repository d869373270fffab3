#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_sk.py > gpurun_out/r4_gsk_tests.log 2>&1 || { echo GSKFAIL; tail -40 gpurun_out/r4_gsk_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_gsk_tests.log | tail -2
timeout -k 10 600 python -u scripts/exp/gemm_sk_bench.py --grid > gpurun_out/r4_gsk_bench.jsonl 2> gpurun_out/r4_gsk_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r4_gsk_bench.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4_gsk_bench.jsonl"):
    d = json.loads(l)
    print(f"{d['shape']:>8} M={d['M']:>5} blas={d['hipblaslt_us']:>7} ({d['hipblaslt_pf']}) plan{d['plan']}={d['plan_us']:>7} ({d['plan_pf']}) best{d.get('best')} ({d.get('best_pf')})")
PY
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_engine_gpu.py tests/test_tp_gpu.py tests/test_custom_allreduce_gpu.py -k "prefill3 or hub_server or follower_hang or custom_allreduce" > gpurun_out/r4_g2_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g2_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r4_g2_tests.log | tail -14
