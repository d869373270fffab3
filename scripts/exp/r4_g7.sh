#!/bin/bash
# Round 4: TP bitwise emulation test, config-5 per-rank projection, TTS-on hub
# cost, encoder-on-split-K and dedicated H2D stager stream A/Bs, decode-step anatomy.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py tests/test_engine_gpu.py -k "bitwise or placed_stream or prefill_hw" > gpurun_out/r4_g7_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g7_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g7_tests.log | tail -2
timeout -k 10 400 python -u scripts/config5_projection.py > gpurun_out/r4_config5_projection.json 2> gpurun_out/r4_config5_projection.err || { echo C5FAIL; tail -20 gpurun_out/r4_config5_projection.err; exit 1; }
tail -c 1500 gpurun_out/r4_config5_projection.json
hub() {  # name args...
  local name=$1; shift
  timeout -k 10 400 python bench.py --mode hub --served-dp --gpus 1 --steps 20 --warmup 5 "$@" > gpurun_out/hub_$name.json 2> gpurun_out/hub_$name.err || { echo "FAIL hub $name"; tail -20 gpurun_out/hub_$name.err; exit 1; }
  grep '^{' gpurun_out/hub_$name.json | tail -1 | cut -c1-600
}
hub notts && hub tts --tts || exit 1
ab() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "FAIL $name"; tail -20 gpurun_out/ab_$name.err; exit 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
ph = d["phase_ms_per_step"]
print(f"{sys.argv[1]:>12} utt/s={d['value']:.3f} e2e={d['ms_per_added_command_e2e_marginal']} prefill={ph['llm_prefill']} decode={ph['llm_decode']} stt={ph['stt']}", flush=True)
PY
}
ab base LOQA_X=0 && ab encsk LOQA_ENC_SK=1 && ab stager1 LOQA_STAGER_STREAM=1 && \
ab base2 LOQA_X=0 && ab encskb LOQA_ENC_SK=1 && ab stager1b LOQA_STAGER_STREAM=1 || exit 1
STEPS=10 WARMUP=3 PROF_TIMEOUT=400 bash scripts/prof_bench.sh
