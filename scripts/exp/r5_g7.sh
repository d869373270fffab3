# fused qkv + attention with sc1 loads (no acquire fence): tests, isolated
# cost, pipeline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_fused_qkv_attn.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/g7_fqa_tests.txt 2>&1 || exit 11
timeout -k 10 300 python -u scripts/exp/fused_qkv_attn_bench.py > gpurun_out/g7_fqa_bench.jsonl 2>&1 || exit 12
AB="f0|LOQA_FUSE_QKV_ATTN=0;f1|LOQA_FUSE_QKV_ATTN=1" bash scripts/exp/bench_ab.sh > gpurun_out/g7_ab.txt 2>&1 || exit 13
echo done
