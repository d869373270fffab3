#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py tests/test_gemm_sk.py tests/test_kernels_gpu.py -k "prefill3 or encoder_sk or vits or expand" > gpurun_out/r4_g6_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g6_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g6_tests.log | tail -2
ab() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "FAIL $name"; tail -20 gpurun_out/ab_$name.err; exit 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
ls, ph = d["llm_stats"], d["phase_ms_per_step"]
print(f"{sys.argv[1]:>12} utt/s={d['value']:.3f} e2e={d['ms_per_added_command_e2e_marginal']} prefill={ph['llm_prefill']} decode={ph['llm_decode']} steps={ph['llm_decode_steps']} passes={ls.get('prefill_passes')} stt={ph['stt']} enc={ph['stt_encode']}", flush=True)
PY
}
ab base LOQA_X=0 && ab p3 LOQA_PREFILL3=1 && ab p3m2 LOQA_PREFILL3=2 && ab encsk LOQA_ENC_SK=1 && ab both LOQA_PREFILL3=1 LOQA_ENC_SK=1 && \
ab base2 LOQA_X=0 && ab p3b LOQA_PREFILL3=1 && ab encskb LOQA_ENC_SK=1 && ab bothb LOQA_PREFILL3=1 LOQA_ENC_SK=1
