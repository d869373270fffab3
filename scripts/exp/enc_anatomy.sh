# Whisper-large-v3 admission (log-mel + encoder + cross-K/V) at batch 1:
# per-encode kernel anatomy from a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/encprof1
ENC_BS=1 ENC_ITERS=12 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/encprof1 -o enc -- python -u scripts/exp/enc_prof.py > gpurun_out/enc1.log 2>&1 || exit 11
K=$(ls gpurun_out/encprof1/*kernel_trace.csv gpurun_out/encprof1/*/*kernel_trace.csv 2>/dev/null | head -1)
python scripts/exp/tail_anatomy.py "$K" --steps 8 --marker logmel_kernel > gpurun_out/enc1_anatomy.txt 2>&1 || exit 12
rm -rf gpurun_out/encprof1
cat gpurun_out/enc1.log | grep B1
echo done
