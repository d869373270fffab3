#!/bin/bash
# kernel trace of scripts/exp/prefill_prof.py (isolated 8B prefills of ~318 tokens)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/ppf
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ppf -o run -- python scripts/exp/prefill_prof.py > gpurun_out/ppf.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/ppf.log; [ $rc = 0 ] || exit $rc
K=$(ls gpurun_out/ppf/*kernel_trace.csv gpurun_out/ppf/*/*kernel_trace.csv 2>/dev/null | head -1)
gzip -c "$K" > gpurun_out/ppf_trace.csv.gz; rm -rf gpurun_out/ppf
