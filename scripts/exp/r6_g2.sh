# decode attention forms (4-wave / 8-wave single pass / prefetch) + deep
# prefetch / qkv split for the config-5 rank step; kernel numerics first
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "grouped or attn_decode" > gpurun_out/g2_tests.txt 2>&1 || { tail -30 gpurun_out/g2_tests.txt; exit 11; }
tail -2 gpurun_out/g2_tests.txt
run() {
  label=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g2_c5_$label.json 2> gpurun_out/g2_c5_$label.err || { tail -5 gpurun_out/g2_c5_$label.err; exit 12; }
  python - "$label" gpurun_out/g2_c5_$label.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"{sys.argv[1]:>14}: step {d['rank_step_ms_local_collectives']:.3f} ms, projected {d['projected_ms_per_added_command']}")
PY
}
run base X=1
run sk512 LOQA_LLM_ATTN_SPLIT_KEYS=512
run sk512pf LOQA_LLM_ATTN_SPLIT_KEYS=512 LOQA_ATTN_PF_MIN_KEYS=256
run sk512w8 LOQA_LLM_ATTN_SPLIT_KEYS=512 LOQA_ATTN8_MIN_KEYS=256
run sk256w8 LOQA_LLM_ATTN_SPLIT_KEYS=256 LOQA_ATTN8_MIN_KEYS=256
run deep8 LOQA_FUSED_DEEP=8
run deep2 LOQA_FUSED_DEEP=2
run qkvS2 "LOQA_FSPLIT_OVERRIDE=rope:1280x8192:M16=2,1,1"
run qkvS4 "LOQA_FSPLIT_OVERRIDE=rope:1280x8192:M16=4,2,1"
run base2 X=2
echo done
