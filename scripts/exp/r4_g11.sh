#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/exp/prefill_m_sweep.py > gpurun_out/r4_prefill_m_sweep.jsonl 2> gpurun_out/r4_prefill_m_sweep.err || { echo FAIL; tail -20 gpurun_out/r4_prefill_m_sweep.err; exit 1; }
cat gpurun_out/r4_prefill_m_sweep.jsonl
