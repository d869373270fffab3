# prologue-item launches (gemm_skinny.hip PRO): TP bitwise tests, config-5
# rank step with / without, anatomy; attention forms; isolated GEMM counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_tp_gpu.py -m gpu -k "prologue" > gpurun_out/g4_tests_pro.txt 2>&1 || { tail -40 gpurun_out/g4_tests_pro.txt; exit 11; }
tail -4 gpurun_out/g4_tests_pro.txt
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py -m gpu -k "not prologue" > gpurun_out/g4_tests_tp.txt 2>&1 || { tail -40 gpurun_out/g4_tests_tp.txt; exit 12; }
tail -8 gpurun_out/g4_tests_tp.txt
run() {
  label=$1; shift
  env "$@" timeout -k 10 300 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g4_c5_$label.json 2> gpurun_out/g4_c5_$label.err || { tail -5 gpurun_out/g4_c5_$label.err; exit 13; }
  python - "$label" gpurun_out/g4_c5_$label.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"{sys.argv[1]:>14}: step {d['rank_step_ms_local_collectives']:.3f} ms, projected {d['projected_ms_per_added_command']}")
PY
}
run pro X=1
run nopro LOQA_TP_PROLOGUE=0
run pro_sk512 LOQA_LLM_ATTN_SPLIT_KEYS=512
run nopro_sk512 LOQA_TP_PROLOGUE=0 LOQA_LLM_ATTN_SPLIT_KEYS=512
run pro_sk256 LOQA_LLM_ATTN_SPLIT_KEYS=256
run nopro_sk512w8 LOQA_TP_PROLOGUE=0 LOQA_LLM_ATTN_SPLIT_KEYS=512 LOQA_ATTN8_MIN_KEYS=256
run nopro_sk512pf LOQA_TP_PROLOGUE=0 LOQA_LLM_ATTN_SPLIT_KEYS=512 LOQA_ATTN_PF_MIN_KEYS=256
run pro2 X=2
rm -rf gpurun_out/g4_c5prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g4_c5prof -o c5 -- python -u scripts/config5_projection.py --iters 10 --prefill-rows 0 > gpurun_out/g4_c5prof.log 2>&1 || { tail -20 gpurun_out/g4_c5prof.log; exit 14; }
f=$(ls gpurun_out/g4_c5prof/c5_kernel_trace.csv gpurun_out/g4_c5prof/*/c5_kernel_trace.csv 2>/dev/null | head -1)
python scripts/decode_steps.py "$f" tp > gpurun_out/g4_c5_anatomy.txt 2>&1; cat gpurun_out/g4_c5_anatomy.txt
rm -rf gpurun_out/g4_c5prof
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "grouped or attn_decode" > gpurun_out/g4_tests_attn.txt 2>&1 || { tail -30 gpurun_out/g4_tests_attn.txt; exit 15; }
tail -2 gpurun_out/g4_tests_attn.txt
bash scripts/pmc_gemm.sh > gpurun_out/g4_pmc.log 2>&1; tail -14 gpurun_out/g4_pmc.log
echo done
