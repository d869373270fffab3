# MMS-TTS-size VITS checkpoint: GPU test, then ours vs transformers timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_vits_checkpoint.py -m gpu > gpurun_out/g28_tests.txt 2>&1 || { tail -30 gpurun_out/g28_tests.txt; exit 1; }
tail -3 gpurun_out/g28_tests.txt
timeout -k 10 400 python -u scripts/exp/vits_mms_bench.py --iters 10 > gpurun_out/g28_mms_bench.jsonl 2> gpurun_out/g28_mms_bench.err || { tail -20 gpurun_out/g28_mms_bench.err; exit 1; }
cat gpurun_out/g28_mms_bench.jsonl
