# Whisper-large-v3 admission work (log-mel + encoder + cross-K/V) alone:
# time per micro-batch, then a kernel trace of it
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/exp/enc_prof.py > gpurun_out/g11_enc.json 2>&1 || exit 11
rm -rf gpurun_out/encprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/encprof -o enc -- python -u scripts/exp/enc_prof.py > gpurun_out/g11_encprof.log 2>&1 || exit 12
S=$(ls gpurun_out/encprof/*kernel_stats.csv gpurun_out/encprof/*/*kernel_stats.csv 2>/dev/null | head -1)
python scripts/kernel_summary.py "$S" 25 > gpurun_out/g11_enc_kernels.txt 2>&1 || exit 13
rm -rf gpurun_out/encprof
echo done
