# mixed-pass split attention: GPU tests, then the pipeline A/B (LOQA_MIXED_SPLIT_ATTN)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_mixed_attention.py tests/test_engine_gpu.py -k "mixed or chunked or fullsize or llm" -m gpu \
  > gpurun_out/g26_tests.txt 2>&1 || { tail -30 gpurun_out/g26_tests.txt; exit 1; }
tail -3 gpurun_out/g26_tests.txt
AB="s0|LOQA_MIXED_SPLIT_ATTN=0;s1|LOQA_MIXED_SPLIT_ATTN=1;s0b|LOQA_MIXED_SPLIT_ATTN=0;s1b|LOQA_MIXED_SPLIT_ATTN=1;s0c|LOQA_MIXED_SPLIT_ATTN=0;s1c|LOQA_MIXED_SPLIT_ATTN=1" BENCH_ARGS="--steps 20 --warmup 5" bash scripts/exp/bench_ab.sh
