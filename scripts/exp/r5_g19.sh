# VITS at the served hub's batch sizes (1 / 2 phrases) and at 8: time per
# batch, then the per-kernel anatomy of 2-phrase graph replays
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2; do
  timeout -k 10 200 python -u scripts/exp/vits_prof.py --iters 10 --phrases $n > gpurun_out/g21_vits_p$n.json 2>&1 || exit 11
  grep '^{' gpurun_out/g21_vits_p$n.json | cut -c1-200
done
rm -rf gpurun_out/vprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vprof -o v -- python -u scripts/exp/vits_prof.py --iters 10 --phrases 2 > gpurun_out/g21_vprof.log 2>&1 || exit 12
S=$(ls gpurun_out/vprof/*kernel_stats.csv gpurun_out/vprof/*/*kernel_stats.csv 2>/dev/null | head -1)
python scripts/kernel_summary.py "$S" 25 > gpurun_out/g21_vits_kernels.txt 2>&1 || exit 13
rm -rf gpurun_out/vprof
echo done
