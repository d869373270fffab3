#!/bin/bash
# Round 4: the Cijk-free defaults (encoder on split-K, prompt-pass logits on
# the skinny lm_head) - tests, headline bench x2 and its kernel trace; VITS
# graphs vs eager + its kernel trace and counters; counters of the hand-written
# prefill GEMMs in a real prompt pass.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_gemm_sk.py -k "prefill_hw or encoder_sk or skinny_lm_head or vits" > gpurun_out/r4_g8_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g8_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g8_tests.log | tail -2
for n in a b; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench_$n.json 2> gpurun_out/r4_bench_$n.err || { echo BENCHFAIL; tail -20 gpurun_out/r4_bench_$n.err; exit 1; }
  grep '^{' gpurun_out/r4_bench_$n.json | cut -c1-330
done
STEPS=10 WARMUP=3 PROF_TIMEOUT=400 bash scripts/prof_bench.sh > gpurun_out/r4_prof.log 2>&1 || { echo PROFFAIL; tail -20 gpurun_out/r4_prof.log; exit 1; }
grep -c Cijk gpurun_out/kernel_summary.txt || true
head -14 gpurun_out/kernel_summary.txt
timeout -k 10 300 python scripts/exp/vits_prof.py --eager > gpurun_out/r4_vits_eager.json 2> gpurun_out/r4_vits_eager.err || { echo VITSFAIL; tail -20 gpurun_out/r4_vits_eager.err; exit 1; }
timeout -k 10 300 python scripts/exp/vits_prof.py > gpurun_out/r4_vits_graph.json 2> gpurun_out/r4_vits_graph.err || { echo VITSFAIL; tail -20 gpurun_out/r4_vits_graph.err; exit 1; }
cut -c1-400 gpurun_out/r4_vits_eager.json gpurun_out/r4_vits_graph.json
rm -rf gpurun_out/vprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vprof -o run -- python3 scripts/exp/vits_prof.py --iters 3 > gpurun_out/vprof.log 2>&1 || { echo VPROFFAIL; tail -20 gpurun_out/vprof.log; exit 1; }
S=$(ls gpurun_out/vprof/*kernel_stats.csv gpurun_out/vprof/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 scripts/kernel_summary.py "$S" 20 > gpurun_out/r4_vits_kernel_summary.txt 2>&1; head -16 gpurun_out/r4_vits_kernel_summary.txt
rm -rf gpurun_out/vprof
PMC_CMD="python3 scripts/exp/vits_prof.py --iters 2" TAG=vits bash scripts/pmc_bench.sh || exit 1
PMC_CMD="python3 scripts/exp/prefill_prof.py" TAG=prefill bash scripts/pmc_bench.sh || exit 1
