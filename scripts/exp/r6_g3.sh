# (1) config-5 rank step: decode-attention forms, now with the split reaching
# the step (2) isolated 8B decode GEMM counters (3) 8B bench: attention forms
# (4) config 5 at one stream (70B TP=1, no TTS): steps per added command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  label=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g3_c5_$label.json 2> gpurun_out/g3_c5_$label.err || { tail -5 gpurun_out/g3_c5_$label.err; exit 12; }
  python - "$label" gpurun_out/g3_c5_$label.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"{sys.argv[1]:>14}: step {d['rank_step_ms_local_collectives']:.3f} ms, projected {d['projected_ms_per_added_command']}")
PY
}
run base X=1
run sk512 LOQA_LLM_ATTN_SPLIT_KEYS=512
run sk512pf LOQA_LLM_ATTN_SPLIT_KEYS=512 LOQA_ATTN_PF_MIN_KEYS=256
run sk512w8 LOQA_LLM_ATTN_SPLIT_KEYS=512 LOQA_ATTN8_MIN_KEYS=256
run sk256w8 LOQA_LLM_ATTN_SPLIT_KEYS=256 LOQA_ATTN8_MIN_KEYS=256
run sk256 LOQA_LLM_ATTN_SPLIT_KEYS=256
bash scripts/pmc_gemm.sh > gpurun_out/g3_pmc.log 2>&1; tail -12 gpurun_out/g3_pmc.log
bench() {
  label=$1; shift
  env "$@" timeout -k 10 400 python bench.py --mode closed > gpurun_out/g3_b_$label.log 2>&1 || { tail -20 gpurun_out/g3_b_$label.log; exit 13; }
  python - "$label" gpurun_out/g3_b_$label.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
p = d["phase_ms_per_step"]
print(f"{sys.argv[1]:>10}: {d['value']} utt/s, stt {p['stt']} llm {p['llm_total']} dec {p['llm_decode']}/{p['llm_decode_steps']} mixed {p['llm_mixed']}")
PY
}
bench base X=1
bench w8x LOQA_ATTN8_MIN_KEYS=256
bench sk256w8 LOQA_ATTN8_MIN_KEYS=256 LOQA_LLM_ATTN_SPLIT_KEYS=256
bench base2 X=2
timeout -k 10 900 python -u scripts/bench_configs.py --config 5 --streams 1 --no-tts --per-stream 3 --warmup 1 > gpurun_out/g3_c5_1stream.log 2>&1 || { tail -20 gpurun_out/g3_c5_1stream.log; exit 14; }
grep '^{' gpurun_out/g3_c5_1stream.log | cut -c1-700
echo done
