# served hub + VITS + bypass: TTS batching window 3 (default) vs 12 vs 25 ms
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in ${WS:-12 25}; do
  LOQA_TTS_BATCH_WINDOW_MS=$w timeout -k 10 600 python -u bench.py --mode hub --served-dp --tts --steps 8 --warmup 2 --bypass > gpurun_out/g16_tts_w$w.log 2>&1 || exit 11
  echo "w$w $(grep '^{' gpurun_out/g16_tts_w$w.log | tail -1 | cut -c1-120)"
done
echo done
