# fused qkv + attention (ATTD): GPU tests, interleaved bench A/B, and an
# anatomy profile of the fused variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_fused_qkv_attn.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/g4_fqa_tests.txt 2>&1 || exit 11
AB="f0|LOQA_FUSE_QKV_ATTN=0;f1|LOQA_FUSE_QKV_ATTN=1;f0b|LOQA_FUSE_QKV_ATTN=0;f1b|LOQA_FUSE_QKV_ATTN=1" \
  bash scripts/exp/bench_ab.sh > gpurun_out/g4_ab.txt 2>&1 || exit 12
LOQA_FUSE_QKV_ATTN=1 bash scripts/prof_bench.sh > gpurun_out/g4_prof.txt 2>&1 || exit 13
cp gpurun_out/anatomy.txt gpurun_out/g4_anatomy_fused.txt
echo done
