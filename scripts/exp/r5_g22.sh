#!/bin/bash
# gemm_sk deeper-ring layouts 9-11: numerics vs fp32, then the layout x split
# grid on the prompt-pass / encoder shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_sk.py -m gpu > gpurun_out/r5_g22_tests.txt 2>&1 || { tail -30 gpurun_out/r5_g22_tests.txt; exit 1; }
tail -3 gpurun_out/r5_g22_tests.txt
timeout -k 10 900 python -u scripts/exp/gemm_sk_bench.py --grid --ms 300 --wms 1500,3000 \
  > gpurun_out/r5_sk_grid_deep.jsonl 2> gpurun_out/r5_sk_grid_deep.err
rc=$?; tail -c 3000 gpurun_out/r5_sk_grid_deep.jsonl | cut -c1-300; exit $rc
