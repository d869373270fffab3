# served hub with on-GPU VITS speaking every reply, window vs single-relay bypass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --mode hub --served-dp --tts --steps 8 --warmup 2 --bypass > gpurun_out/g14_hub_tts_bypass.log 2>&1 || exit 11
grep '^{' gpurun_out/g14_hub_tts_bypass.log | tail -1 | cut -c1-300
echo done
