#!/bin/bash
# Round 4 check: every GPU test, smoke, headline bench (driver shape) and its profile.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 560 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/smoke.log; exit 1; }
grep -v amdgpu.ids gpurun_out/smoke.log | tail -2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | cut -c1-400
STEPS=10 WARMUP=3 PROF_TIMEOUT=400 bash scripts/prof_bench.sh > gpurun_out/r4_prof_final.log 2>&1 || { echo PROFFAIL; tail -20 gpurun_out/r4_prof_final.log; exit 1; }
head -14 gpurun_out/kernel_summary.txt
cat gpurun_out/anatomy.txt | head -14
