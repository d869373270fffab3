set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/exp/prefill_prof.py || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pprof -o run -- python scripts/exp/prefill_prof.py > gpurun_out/pprof.log 2>&1 || exit $?
S=$(ls gpurun_out/pprof/*kernel_stats.csv gpurun_out/pprof/*/*kernel_stats.csv 2>/dev/null | head -1)
python scripts/kernel_summary.py "$S" 24 > gpurun_out/pprof_summary.txt
rm -rf gpurun_out/pprof
bash scripts/bench_sweep.sh xl: noxl:LOQA_TUNE_XL=0
