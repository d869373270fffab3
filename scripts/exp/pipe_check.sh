set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "llm" > gpurun_out/llm_gpu_tests.log 2>&1
rc=$?; tail -12 gpurun_out/llm_gpu_tests.log; [ $rc = 0 ] || exit $rc
bash scripts/bench_sweep.sh pipe: nopipe:LOQA_LLM_PIPELINE=0
