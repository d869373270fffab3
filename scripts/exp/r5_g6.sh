# isolated fused qkv + attention cost (workers = items vs GEMM blocks only),
# then config 5 (lean all-reduce publish through the TP tests, projection)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/exp/fused_qkv_attn_bench.py > gpurun_out/g6_fqa_bench.jsonl 2>&1 || exit 11
LOQA_ATTD_WORKERS=0 timeout -k 10 300 python -u scripts/exp/fused_qkv_attn_bench.py > gpurun_out/g6_fqa_bench_w0.jsonl 2>&1 || exit 12
bash scripts/exp/r5_g5.sh > gpurun_out/g6_c5.txt 2>&1 || exit 13
echo done
