# served hub (default) vs closed loop, three more interleaved pairs on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
bench() {
  label=$1; shift
  timeout -k 10 400 python bench.py --window-steps 0 "$@" > gpurun_out/g13_$label.log 2>&1 || { tail -20 gpurun_out/g13_$label.log; exit 13; }
  python - "$label" gpurun_out/g13_$label.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0])
p = d["phase_ms_per_step"]
print(f"{sys.argv[1]:>8}: {d['value']} utt/s {d['config']['mode']}, ms/added {d['ms_per_added_command_e2e_marginal']}, stt {p['stt']} llm {p['llm_total']}")
PY
}
bench hub1
bench closed1 --mode closed
bench hub2
bench closed2 --mode closed
bench hub3
bench closed3 --mode closed
echo benches done
