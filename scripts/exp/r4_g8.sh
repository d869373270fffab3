#!/bin/bash
# Round 4: VITS graphs vs eager + its kernel trace and counters; counters of the
# hand-written prefill GEMMs in a real prompt pass; headline bench kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/exp/vits_prof.py --eager > gpurun_out/r4_vits_eager.json 2> gpurun_out/r4_vits_eager.err || { echo VITSFAIL; tail -20 gpurun_out/r4_vits_eager.err; exit 1; }
timeout -k 10 300 python scripts/exp/vits_prof.py > gpurun_out/r4_vits_graph.json 2> gpurun_out/r4_vits_graph.err || { echo VITSFAIL; tail -20 gpurun_out/r4_vits_graph.err; exit 1; }
cut -c1-400 gpurun_out/r4_vits_eager.json gpurun_out/r4_vits_graph.json
rm -rf gpurun_out/vprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vprof -o run -- python3 scripts/exp/vits_prof.py --iters 3 > gpurun_out/vprof.log 2>&1 || { echo VPROFFAIL; tail -20 gpurun_out/vprof.log; exit 1; }
S=$(ls gpurun_out/vprof/*kernel_stats.csv gpurun_out/vprof/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 scripts/kernel_summary.py "$S" 20 > gpurun_out/r4_vits_kernel_summary.txt 2>&1; head -25 gpurun_out/r4_vits_kernel_summary.txt
rm -rf gpurun_out/vprof
PMC_CMD="python3 scripts/exp/vits_prof.py --iters 2" TAG=vits bash scripts/pmc_bench.sh || exit 1
LOQA_PREFILL3=1 PMC_CMD="python3 scripts/exp/prefill_prof.py" TAG=prefill3 bash scripts/pmc_bench.sh || exit 1
