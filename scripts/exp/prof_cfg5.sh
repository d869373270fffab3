#!/bin/bash
# kernel stats of config 5 (Whisper-large-v3 + Llama-3-70B compact + VITS, TP=1)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/p5
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p5 -o run -- python scripts/bench_configs.py --config 5 > gpurun_out/p5.log 2>&1
rc=$?; echo "rc=$rc"; grep "^{" gpurun_out/p5.log | cut -c1-400; [ $rc = 0 ] || exit $rc
S=$(ls gpurun_out/p5/*kernel_stats.csv gpurun_out/p5/*/*kernel_stats.csv 2>/dev/null | head -1)
python scripts/kernel_summary.py "$S" 30 > gpurun_out/cfg5_kernel_summary.txt 2>&1
K=$(ls gpurun_out/p5/*kernel_trace.csv gpurun_out/p5/*/*kernel_trace.csv 2>/dev/null | head -1)
gzip -c "$K" > gpurun_out/p5_trace.csv.gz; rm -rf gpurun_out/p5
head -30 gpurun_out/cfg5_kernel_summary.txt
