#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_sk.py -k "gemm_ws or gemm_sk_gpu or deterministic" > gpurun_out/r4_g5_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g5_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g5_tests.log | tail -2
timeout -k 10 600 python -u scripts/exp/gemm_sk_bench.py --ms 300,600,1200 --wms 1500,3000 --grid > gpurun_out/r4_g5_bench.jsonl 2> gpurun_out/r4_g5_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r4_g5_bench.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4_g5_bench.jsonl"):
    d = json.loads(l)
    g = sorted(d["grid"].items(), key=lambda kv: kv[1])[:3]
    print(f"{d['shape']:>8} M={d['M']:>5} blas={d['hipblaslt_us']:>7} sk{d['plan']}={d['plan_us']:>7} ws={d['ws_us']} best={g}")
PY
