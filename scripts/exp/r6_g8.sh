# served-hub overhead vs the closed loop, one box, interleaved: PCM stream-in
# and the predictive bridge off / on
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bench() {
  label=$1; envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --window-steps 0 "$@" > gpurun_out/g8_$label.log 2>&1 || { tail -20 gpurun_out/g8_$label.log; exit 13; }
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
echo benches done
# official config-5 projection (default 7-launch TP step) and its rank-step anatomy
timeout -k 10 300 python -u scripts/config5_projection.py --iters 30 --steps-per-command-1stream 25.1 --stt-ms-per-command-1stream 12.3 > gpurun_out/g8_c5proj.json 2> gpurun_out/g8_c5proj.err || { tail -5 gpurun_out/g8_c5proj.err; exit 14; }
rm -rf gpurun_out/g8_prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g8_prof -o c5 -- python -u scripts/config5_projection.py --iters 10 --prefill-rows 0 > gpurun_out/g8_prof.log 2>&1 || { tail -20 gpurun_out/g8_prof.log; exit 15; }
f=$(ls gpurun_out/g8_prof/c5_kernel_trace.csv gpurun_out/g8_prof/*/c5_kernel_trace.csv 2>/dev/null | head -1)
python scripts/decode_steps.py "$f" tp > gpurun_out/g8_anat_c5.txt 2>&1; head -12 gpurun_out/g8_anat_c5.txt
rm -rf gpurun_out/g8_prof
echo alldone
