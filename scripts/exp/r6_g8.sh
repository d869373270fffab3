# served-hub overhead vs the closed loop, one box, interleaved: PCM stream-in
# and the predictive bridge off / on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bench() {
  label=$1; shift
  env "$@" timeout -k 10 400 python bench.py --window-steps 0 > gpurun_out/g8_$label.log 2>&1 || { tail -20 gpurun_out/g8_$label.log; exit 13; }
  python - "$label" gpurun_out/g8_$label.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
p = d["phase_ms_per_step"]
print(f"{sys.argv[1]:>10}: {d['value']} utt/s {d['config']['mode']}, stt {p['stt']} llm {p['llm_total']} dec {p['llm_decode']}/{p['llm_decode_steps']} mixed {p['llm_mixed']}")
PY
}
bench hub X=1
bench closed X=1 --mode closed
bench hub_nosi LOQA_PCM_STREAM_IN=0
bench hub_nobr LOQA_BENCH_NO_BRIDGE=1
bench hub2 X=2
bench closed2 X=2 --mode closed
bench hub_nosi2 LOQA_PCM_STREAM_IN=0
bench hub_nobr2 LOQA_BENCH_NO_BRIDGE=1
echo done
