#!/bin/bash
# kernel stats of scripts/exp/step_cost_by_t.py (decode steps at T = 8..128)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/pst
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pst -o run -- python scripts/exp/step_cost_by_t.py > gpurun_out/pst.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc = 0 ] || exit $rc
K=$(ls gpurun_out/pst/*kernel_trace.csv gpurun_out/pst/*/*kernel_trace.csv 2>/dev/null | head -1)
gzip -c "$K" > gpurun_out/pst_trace.csv.gz; rm -rf gpurun_out/pst
