# 8B headline bench (closed loop, 20 steps): decode-attention forms and the qkv
# layout; then config 5 at one stream (70B TP=1, no TTS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bench() {
  label=$1; shift
  env "$@" timeout -k 10 400 python bench.py --mode closed > gpurun_out/g5_b_$label.log 2>&1 || { tail -20 gpurun_out/g5_b_$label.log; exit 13; }
  python - "$label" gpurun_out/g5_b_$label.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
p = d["phase_ms_per_step"]
print(f"{sys.argv[1]:>10}: {d['value']} utt/s, stt {p['stt']} llm {p['llm_total']} dec {p['llm_decode']}/{p['llm_decode_steps']} mixed {p['llm_mixed']}")
PY
}
timeout -k 10 400 python bench.py > gpurun_out/g5_hub.log 2>&1 || { tail -20 gpurun_out/g5_hub.log; exit 12; }
python - gpurun_out/g5_hub.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
p = d["phase_ms_per_step"]
print(f"   hub(default): {d['value']} utt/s mode {d['config']['mode']}, stt {p['stt']} llm {p['llm_total']} "
      f"dec {p['llm_decode']}/{p['llm_decode_steps']} mixed {p['llm_mixed']}, events {d['hub']['voice_events']}, "
      f"window {d['window_300ms']}")
PY
bench base X=1
bench w8x LOQA_ATTN8_MIN_KEYS=256
bench pfx LOQA_ATTN_PF_MIN_KEYS=256
bench sk256w8 LOQA_ATTN8_MIN_KEYS=256 LOQA_LLM_ATTN_SPLIT_KEYS=256
bench qkvrt1 "LOQA_FSPLIT_OVERRIDE=rope:6144x4096:M16=1,1,1"
bench base2 X=2
timeout -k 10 900 python -u scripts/bench_configs.py --config 5 --streams 1 --no-tts --per-stream 3 --warmup 1 > gpurun_out/g5_c5_1stream.log 2>&1 || { tail -20 gpurun_out/g5_c5_1stream.log; exit 14; }
grep '^{' gpurun_out/g5_c5_1stream.log | cut -c1-900
echo done
