#!/bin/bash
# Round 4: chunk-size sweep of the mixed prompt passes (40 timed steps, interleaved).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/exp/gemm_sk_bench.py --ms 64,128,192,256 --wms 1500 --grid --only qkv,o,gu,down > gpurun_out/r4_gemm_small_m.jsonl 2> gpurun_out/r4_gemm_small_m.err || { echo GRIDFAIL; tail -20 gpurun_out/r4_gemm_small_m.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r4_gemm_small_m.jsonl"):
    d = json.loads(l)
    g = sorted(d["grid"].items(), key=lambda kv: kv[1])[:3]
    print(f"{d['shape']:>5} M={d['M']:>4} blas={d['hipblaslt_us']:>6} plan{d['plan']}={d['plan_us']:>6} ws={d['ws_us']} best={g}")
PY
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
