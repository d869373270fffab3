#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_sk.py -k "gemm_ws" > gpurun_out/r4_gws_tests.log 2>&1 || { echo GWSFAIL; tail -40 gpurun_out/r4_gws_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_gws_tests.log | tail -2
timeout -k 10 600 python -u scripts/exp/gemm_sk_bench.py --ms 300,600 --wms 1500,3000 > gpurun_out/r4_gws_bench.jsonl 2> gpurun_out/r4_gws_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r4_gws_bench.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4_gws_bench.jsonl"):
    d = json.loads(l)
    print(f"{d['shape']:>8} M={d['M']:>5} blas={d['hipblaslt_us']:>7} sk{d['plan']}={d['plan_us']:>7} ws={d['ws_us']}")
PY
