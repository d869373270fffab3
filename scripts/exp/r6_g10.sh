# STT pipeline host timing under the default bench (where the Whisper
# step-to-step gap comes from)
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --window-steps 0 > gpurun_out/g10_bench.log 2>&1 || { tail -20 gpurun_out/g10_bench.log; exit 3; }
python - gpurun_out/g10_bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
s = d["stt_stats"]
n = max(1, s["pl_steps"])
print("value", d["value"], "stt", d["phase_ms_per_step"]["stt"])
print({k: s[k] for k in s if not isinstance(s[k], float)})
for k in ("gpu_wait_s", "pl_launch_s", "pl_replay_s", "encode_s"):
    print(k, round(s.get(k, 0.0), 3), "s total,", round(1e6 * s.get(k, 0.0) / n, 1), "us per step")
PY
echo alldone
