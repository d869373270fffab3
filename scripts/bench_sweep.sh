#!/bin/bash
# Run bench.py once per "NAME:ENV=VAL,ENV=VAL" variant (each under its own time
# limit); prints one summary line per variant, stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  args=()
  if [ "$envs" != "$spec" ] && [ -n "$envs" ]; then IFS=',' read -ra args <<< "$envs"; fi
  env "${args[@]}" timeout -k 10 ${BENCH_TIMEOUT:-240} python bench.py ${BENCH_ARGS:-} > gpurun_out/sweep_$name.log 2>&1
  rc=$?
  line=$(grep '^{' gpurun_out/sweep_$name.log | tail -1)
  python - "$name" "$line" <<'PY'
import json, sys
name, line = sys.argv[1], sys.argv[2]
try:
    d = json.loads(line)
    ph = d.get("phase_ms_per_step", {})
    ls = d.get("llm_stats", {})
    print(f"{name:14s} utt/s {d['value']:7.3f}  ms/added {d.get('ms_per_added_command_e2e_marginal')}  stt {ph.get('stt')}  "
          f"prefill {ph.get('llm_prefill')}  decode_steps {ls.get('decode_steps')}  "
          f"ms/step {1e3*ls.get('decode_s',0)/max(1,ls.get('decode_steps',1)):.2f}")
except Exception as e:
    print(name, "no result", e)
PY
  [ $rc = 0 ] || { echo "$name rc=$rc - stopping"; tail -5 gpurun_out/sweep_$name.log; exit $rc; }
done
