#!/bin/bash
# Round 4: LDS-staged conv1d (VITS) - kernel tests vs fp32 torch, VITS model
# tests, timing graphs vs eager, counters, served hub with TTS.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "conv or vits" > gpurun_out/r4_g14_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g14_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g14_tests.log | tail -2
timeout -k 10 300 python scripts/exp/vits_prof.py --eager > gpurun_out/r4_vits_eager3.json 2> gpurun_out/r4_vits_eager3.err || { echo VITSFAIL; tail -20 gpurun_out/r4_vits_eager3.err; exit 1; }
timeout -k 10 300 python scripts/exp/vits_prof.py > gpurun_out/r4_vits_graph3.json 2> gpurun_out/r4_vits_graph3.err || { echo VITSFAIL; tail -20 gpurun_out/r4_vits_graph3.err; exit 1; }
cut -c1-300 gpurun_out/r4_vits_eager3.json gpurun_out/r4_vits_graph3.json
PMC_CMD="python3 scripts/exp/vits_prof.py --iters 2" TAG=vits3 bash scripts/pmc_bench.sh > gpurun_out/pmc_vits3.log 2>&1 || { echo PMCFAIL; exit 1; }
grep -E "conv1d|kernel " gpurun_out/pmc_vits3.txt || true
timeout -k 10 400 python bench.py --mode hub --served-dp --gpus 1 --steps 20 --warmup 5 --tts > gpurun_out/hub_tts3.json 2> gpurun_out/hub_tts3.err || { echo "FAIL hub"; tail -20 gpurun_out/hub_tts3.err; exit 1; }
grep '^{' gpurun_out/hub_tts3.json | tail -1 | cut -c1-200
timeout -k 10 400 python bench.py --mode hub --served-dp --gpus 1 --steps 20 --warmup 5 > gpurun_out/hub_notts3.json 2> gpurun_out/hub_notts3.err || { echo "FAIL hub"; tail -20 gpurun_out/hub_notts3.err; exit 1; }
grep '^{' gpurun_out/hub_notts3.json | tail -1 | cut -c1-200
