# config 5 (Llama-3-70B TP=8 rank): the lean residual all-reduce publish
# (LOQA_CAR_LEAN) through the multi-process TP tests, then the per-rank step
# projection: baseline / lean / lean + fused qkv-attention
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
LOQA_CAR_LEAN=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/g5_tp_lean.txt 2>&1 || exit 11
for v in "base|LOQA_CAR_LEAN=0 LOQA_FUSE_QKV_ATTN=0" "lean|LOQA_CAR_LEAN=1 LOQA_FUSE_QKV_ATTN=0" "lean_attd|LOQA_CAR_LEAN=1 LOQA_FUSE_QKV_ATTN=1"; do
  label="${v%%|*}"; envs="${v#*|}"
  env $envs timeout -k 10 400 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g5_c5_${label}.json 2> gpurun_out/g5_c5_${label}.err || exit 12
  echo "$label $(cat gpurun_out/g5_c5_${label}.json | cut -c1-400)"
done
echo done
