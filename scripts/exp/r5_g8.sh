# config 5 rank step: kernel summary with the lean all-reduce (8 layers)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/c5prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof -o c5 -- python -u scripts/config5_projection.py --iters 20 --layers 80 --prefill-rows 0 > gpurun_out/g8_c5prof.log 2>&1 || exit 11
S=$(ls gpurun_out/c5prof/*kernel_stats.csv gpurun_out/c5prof/*/*kernel_stats.csv 2>/dev/null | head -1)
python scripts/kernel_summary.py "$S" 30 > gpurun_out/g8_c5_kernel_summary.txt 2>&1 || exit 12
K=$(ls gpurun_out/c5prof/*kernel_trace.csv gpurun_out/c5prof/*/*kernel_trace.csv 2>/dev/null | head -1)
python scripts/exp/tail_anatomy.py "$K" --steps 10 > gpurun_out/g8_c5_anatomy.txt 2>&1 || exit 13
rm -rf gpurun_out/c5prof
echo done
