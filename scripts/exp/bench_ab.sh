# A/B benches: each line of $AB is "label|ENV=VAL ENV2=VAL" (empty env = default)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=';' read -ra RUNS <<< "${AB}"
for run in "${RUNS[@]}"; do
  label="${run%%|*}"; envs="${run#*|}"
  env $envs timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > "gpurun_out/ab_${label}.log" 2>&1
  rc=$?
  python3 - "$label" "gpurun_out/ab_${label}.log" <<'PY'
import json, sys
label, path = sys.argv[1], sys.argv[2]
for l in open(path):
    if l.startswith('{"metric"'):
        d = json.loads(l)
        ph = d.get("phase_ms_per_step", {})
        print(label, d["value"], "ms/added", d.get("ms_per_added_command_e2e_marginal"),
              "stt", ph.get("stt"), "prefill", ph.get("llm_prefill"), "decode", ph.get("llm_decode"),
              "steps", ph.get("llm_decode_steps"))
PY
  [ $rc -eq 0 ] || { echo "$label rc=$rc"; exit $rc; }
done
