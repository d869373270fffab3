# served-hub soak: 150 timed steps (1200 utterances) on the default bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python bench.py --steps 150 --warmup 5 --window-steps 0 > gpurun_out/g12_soak.log 2>&1 || { tail -20 gpurun_out/g12_soak.log; exit 4; }
python - gpurun_out/g12_soak.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
h = d["hub"]
print("soak", d["value"], "utt/s", d["steps"], "steps", "ms/added", d["ms_per_added_command_e2e_marginal"],
      "events", h["voice_events"], "timed", h["timed_utterances"], "p50", h["latency_ms_p50"], "p90", h["latency_ms_p90"],
      "match", d["command_count_match_rate"], "ok", d["queue_success_rate"], "errors", h["processor"]["errors"],
      "stt", d["phase_ms_per_step"]["stt"], "llm", d["phase_ms_per_step"]["llm_total"])
PY
echo soakdone
