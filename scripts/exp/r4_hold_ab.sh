#!/bin/bash
# A/B of the prefill coalescing hold (LOQA_PREFILL_HOLD_MS) on the headline bench.
set -o pipefail
export TMPDIR=/tmp
for v in ${HOLDS:-0 20 40 0 20 40}; do
  LOQA_PREFILL_HOLD_MS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/hold_$v.json 2> gpurun_out/hold_$v.err || { echo "FAIL hold=$v"; tail -20 gpurun_out/hold_$v.err; exit 1; }
  python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/hold_{sys.argv[1]}.json").read().strip().splitlines()[-1])
ls = d["llm_stats"]
print(f"hold={sys.argv[1]:>3} utt/s={d['value']:.3f} e2e={d['ms_per_added_command_e2e_marginal']} "
      f"prefill={d['phase_ms_per_step']['llm_prefill']} decode={d['phase_ms_per_step']['llm_decode']} "
      f"steps={d['phase_ms_per_step']['llm_decode_steps']} passes={ls.get('prefill_passes')} "
      f"coalesced={ls.get('prefill_passes_coalesced')} stt={d['phase_ms_per_step']['stt']}", flush=True)
PY
done
