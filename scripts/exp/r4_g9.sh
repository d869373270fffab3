#!/bin/bash
# Round 4: conv1d with grouped loads + batched epilogue loads (VITS) - tests,
# VITS timing / counters, served hub with TTS; config-5 per-rank projection
# (corrected byte count) and its kernel breakdown.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/exp/r4_g10.sh || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "conv or vits or expand" > gpurun_out/r4_g9_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g9_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g9_tests.log | tail -2
timeout -k 10 300 python scripts/exp/vits_prof.py --eager > gpurun_out/r4_vits_eager2.json 2> gpurun_out/r4_vits_eager2.err || { echo VITSFAIL; tail -20 gpurun_out/r4_vits_eager2.err; exit 1; }
timeout -k 10 300 python scripts/exp/vits_prof.py > gpurun_out/r4_vits_graph2.json 2> gpurun_out/r4_vits_graph2.err || { echo VITSFAIL; tail -20 gpurun_out/r4_vits_graph2.err; exit 1; }
cut -c1-300 gpurun_out/r4_vits_eager2.json gpurun_out/r4_vits_graph2.json
PMC_CMD="python3 scripts/exp/vits_prof.py --iters 2" TAG=vits2 bash scripts/pmc_bench.sh > gpurun_out/pmc_vits2.log 2>&1 || { echo PMCFAIL; exit 1; }
grep -E "conv1d|kernel " gpurun_out/pmc_vits2.txt || true
timeout -k 10 400 python bench.py --mode hub --served-dp --gpus 1 --steps 20 --warmup 5 --tts > gpurun_out/hub_tts2.json 2> gpurun_out/hub_tts2.err || { echo "FAIL hub"; tail -20 gpurun_out/hub_tts2.err; exit 1; }
grep '^{' gpurun_out/hub_tts2.json | tail -1 | cut -c1-200
timeout -k 10 400 python -u scripts/config5_projection.py > gpurun_out/r4_config5_projection.json 2> gpurun_out/r4_config5_projection.err || { echo C5FAIL; tail -20 gpurun_out/r4_config5_projection.err; exit 1; }
tail -c 600 gpurun_out/r4_config5_projection.json
rm -rf gpurun_out/c5prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o run -- python3 scripts/config5_projection.py --iters 20 > gpurun_out/c5prof.log 2>&1 || { echo C5PROFFAIL; tail -20 gpurun_out/c5prof.log; exit 1; }
S=$(ls gpurun_out/c5prof/*kernel_stats.csv gpurun_out/c5prof/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 scripts/kernel_summary.py "$S" 25 > gpurun_out/r4_config5_kernel_summary.txt 2>&1; head -30 gpurun_out/r4_config5_kernel_summary.txt
rm -rf gpurun_out/c5prof
