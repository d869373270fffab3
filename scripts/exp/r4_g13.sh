#!/bin/bash
# Round 4: chunked prompt passes - longer interleaved A/B (40 timed steps).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ab() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "FAIL $name"; tail -20 gpurun_out/ab_$name.err; exit 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
ph, ls = d["phase_ms_per_step"], d["llm_stats"]
print(f"{sys.argv[1]:>10} utt/s={d['value']:.3f} e2e={d['ms_per_added_command_e2e_marginal']} decode={ph['llm_decode']} steps={ph['llm_decode_steps']} stt={ph['stt']} llm_total={ph['llm_total']} mixed={ls.get('mixed_steps')} mixed_s={ls.get('mixed_s')} prefill_s={ls.get('prefill_s')}", flush=True)
PY
}
for i in 1 2 3 4; do
  ab c0_$i LOQA_CHUNK_PREFILL=0 && ab c256_$i LOQA_CHUNK_PREFILL=256 && ab c128_$i LOQA_CHUNK_PREFILL=128 || exit 1
done
