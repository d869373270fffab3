#!/bin/bash
# Round 4: chunk-size sweep of the mixed prompt passes (40 timed steps, interleaved).
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
print(f"{sys.argv[1]:>10} utt/s={d['value']:.3f} e2e={d['ms_per_added_command_e2e_marginal']} decode={ph['llm_decode']} steps={ph['llm_decode_steps']} mixed={ph.get('llm_mixed')} mixed_steps={ph.get('llm_mixed_steps')} stt={ph['stt']} llm_total={ph['llm_total']}", flush=True)
PY
}
for i in 1 2 3; do
  ab c192_$i LOQA_CHUNK_PREFILL=192 && ab c256_$i LOQA_CHUNK_PREFILL=256 && ab c320_$i LOQA_CHUNK_PREFILL=320 && ab c512_$i LOQA_CHUNK_PREFILL=512 || exit 1
done
