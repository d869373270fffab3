set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/exp/enc_prof.py || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eprof -o run -- python scripts/exp/enc_prof.py > gpurun_out/eprof.log 2>&1 || exit $?
S=$(ls gpurun_out/eprof/*kernel_stats.csv gpurun_out/eprof/*/*kernel_stats.csv 2>/dev/null | head -1)
python scripts/kernel_summary.py "$S" 20 > gpurun_out/eprof_summary.txt
rm -rf gpurun_out/eprof
