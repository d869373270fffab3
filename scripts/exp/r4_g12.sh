#!/bin/bash
# Round 4: chunked prompt passes riding with the live sequences (mixed steps):
# GPU test and headline A/B over the chunk size (0 = whole prompt passes).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "chunked_prefill" > gpurun_out/r4_g12_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g12_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g12_tests.log | tail -2
ab() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "FAIL $name"; tail -20 gpurun_out/ab_$name.err; exit 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
ph, ls = d["phase_ms_per_step"], d["llm_stats"]
print(f"{sys.argv[1]:>10} utt/s={d['value']:.3f} e2e={d['ms_per_added_command_e2e_marginal']} prefill={ph['llm_prefill']} decode={ph['llm_decode']} steps={ph['llm_decode_steps']} stt={ph['stt']} passes={ls.get('prefill_passes')} mixed={ls.get('mixed_steps')}", flush=True)
PY
}
ab c0 LOQA_CHUNK_PREFILL=0 && ab c512 LOQA_CHUNK_PREFILL=512 && ab c256 LOQA_CHUNK_PREFILL=256 && \
ab c0b LOQA_CHUNK_PREFILL=0 && ab c512b LOQA_CHUNK_PREFILL=512 && ab c256b LOQA_CHUNK_PREFILL=256 || exit 1
