#!/bin/bash
# Round 4: prompt-pass o / down as prefill-GEMM f32 slabs (LOQA_PREFILL_SLABS=1)
# vs the split-K tiled GEMM adding in-launch: test, isolated prompt-pass time,
# headline A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "prefill_hw" > gpurun_out/r4_g10_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r4_g10_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4_g10_tests.log | tail -2
for v in 1 0; do
  LOQA_PREFILL_SLABS=$v timeout -k 10 300 python scripts/exp/prefill_prof.py > gpurun_out/pf_slabs$v.json 2> gpurun_out/pf_slabs$v.err || { echo PFFAIL; tail -20 gpurun_out/pf_slabs$v.err; exit 1; }
  echo "slabs=$v $(tail -1 gpurun_out/pf_slabs$v.json)"
done
ab() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "FAIL $name"; tail -20 gpurun_out/ab_$name.err; exit 1; }
  python - "$name" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
ph = d["phase_ms_per_step"]
print(f"{sys.argv[1]:>12} utt/s={d['value']:.3f} e2e={d['ms_per_added_command_e2e_marginal']} prefill={ph['llm_prefill']} decode={ph['llm_decode']} stt={ph['stt']} enc={ph['stt_encode']}", flush=True)
PY
}
ab slabs1 LOQA_PREFILL_SLABS=1 && ab slabs0 LOQA_PREFILL_SLABS=0 && ab slabs1b LOQA_PREFILL_SLABS=1 && ab slabs0b LOQA_PREFILL_SLABS=0 || exit 1
