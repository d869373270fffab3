#!/bin/bash
# rocprofv3 kernel trace of a short bench run + per-step anatomy of both decoders.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps ${STEPS:-8} --warmup ${WARMUP:-2} ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?
echo "profile rc=$rc"
grep '^{' gpurun_out/prof.log | cut -c1-300
[ $rc = 0 ] || exit $rc
K=$(ls gpurun_out/prof/*kernel_trace.csv gpurun_out/prof/*/*kernel_trace.csv 2>/dev/null | head -1)
S=$(ls gpurun_out/prof/*kernel_stats.csv gpurun_out/prof/*/*kernel_stats.csv 2>/dev/null | head -1)
{ python scripts/decode_steps.py "$K" llm; python scripts/decode_steps.py "$K" stt; } > gpurun_out/anatomy.txt 2>&1
cat gpurun_out/anatomy.txt
python scripts/kernel_summary.py "$S" 25 > gpurun_out/kernel_summary.txt 2>&1 || true
python scripts/timeline.py "$K" > gpurun_out/timeline.txt 2>&1 || true
cp "$S" gpurun_out/kernel_stats.csv
gzip -c "$K" > gpurun_out/kernel_trace.csv.gz
rm -rf gpurun_out/prof
python scripts/busy.py gpurun_out/kernel_trace.csv.gz 1.5 1.0 > gpurun_out/busy.txt 2>&1; cat gpurun_out/busy.txt
