#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_tp_gpu.py tests/test_gemm_sk.py -k "follower_hang or encoder_sk" > gpurun_out/r4_g3_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g3_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r4_g3_tests.log | tail -6
ab() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "FAIL $name"; tail -20 gpurun_out/ab_$name.err; exit 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
ls, ph = d["llm_stats"], d["phase_ms_per_step"]
print(f"{sys.argv[1]:>12} utt/s={d['value']:.3f} e2e={d['ms_per_added_command_e2e_marginal']} prefill={ph['llm_prefill']} decode={ph['llm_decode']} steps={ph['llm_decode_steps']} passes={ls.get('prefill_passes')} coal={ls.get('prefill_passes_coalesced')} stt={ph['stt']}", flush=True)
PY
}
ab base LOQA_X=0 && ab hold25 LOQA_PREFILL_HOLD_MS=25 && ab p3m2 LOQA_PREFILL3=2 && ab hold50 LOQA_PREFILL_HOLD_MS=50 && ab base2 LOQA_X=0 && ab hold25b LOQA_PREFILL_HOLD_MS=25 && ab p3m2b LOQA_PREFILL3=2
