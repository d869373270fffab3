# prologue gate poll back-off sweep + decode-grid cap, config-5 rank step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  label=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g7_c5_$label.json 2> gpurun_out/g7_c5_$label.err || { tail -5 gpurun_out/g7_c5_$label.err; exit 13; }
  python - "$label" gpurun_out/g7_c5_$label.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"{sys.argv[1]:>14}: step {d['rank_step_ms_local_collectives']:.3f} ms, projected {d['projected_ms_per_added_command']}")
PY
}
run nopro X=1
run pro_0_1 LOQA_TP_PROLOGUE=1 LOQA_PRO_SLEEP0=0 LOQA_PRO_SLEEP=1
run pro_2_4 LOQA_TP_PROLOGUE=1 LOQA_PRO_SLEEP0=2 LOQA_PRO_SLEEP=4
run pro_1_2 LOQA_TP_PROLOGUE=1 LOQA_PRO_SLEEP0=1 LOQA_PRO_SLEEP=2
run pro_4_8 LOQA_TP_PROLOGUE=1 LOQA_PRO_SLEEP0=4 LOQA_PRO_SLEEP=8
run nopro_cap512 LOQA_LLM_MAX_WGS=512
run nopro_b X=2
rm -rf gpurun_out/g7_prof
LOQA_TP_PROLOGUE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g7_prof -o c5 -- python -u scripts/config5_projection.py --iters 10 --prefill-rows 0 > gpurun_out/g7_prof.log 2>&1 || { tail -20 gpurun_out/g7_prof.log; exit 14; }
f=$(ls gpurun_out/g7_prof/c5_kernel_trace.csv gpurun_out/g7_prof/*/c5_kernel_trace.csv 2>/dev/null | head -1)
python scripts/decode_steps.py "$f" tp > gpurun_out/g7_anat_pro.txt 2>&1; head -8 gpurun_out/g7_anat_pro.txt
rm -rf gpurun_out/g7_prof
echo done
