#!/bin/bash
# Round 4: small-row projection choices (LOQA_PROJ_SMALLM) with 320-token chunks; chunk 384.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_gemm_sk.py -k "chunked_prefill or prefill_hw or gemm_sk_gpu" > gpurun_out/r4_g16_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g16_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g16_tests.log | tail -2
timeout -k 10 300 python scripts/exp/prefill_m_sweep.py > gpurun_out/r4_prefill_m_sweep2.jsonl 2>&1 || { echo SWEEPFAIL; exit 1; }
tail -1 gpurun_out/r4_prefill_m_sweep2.jsonl
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
  ab sm1_$i LOQA_PROJ_SMALLM=1 && ab sm0_$i LOQA_PROJ_SMALLM=0 && ab c384_$i LOQA_CHUNK_PREFILL=384 || exit 1
done
