set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_decode.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "xl" > gpurun_out/xl_tests.log 2>&1
rc=$?; tail -5 gpurun_out/xl_tests.log; [ $rc = 0 ] || exit $rc
LOQA_TUNE_XL=0 LOQA_LOG_STREAMS=1 timeout -k 10 240 python bench.py > gpurun_out/b_noxl.log 2>&1 || exit $?
grep streams gpurun_out/b_noxl.log; grep '^{' gpurun_out/b_noxl.log | cut -c1-150
LOQA_LOG_STREAMS=1 timeout -k 10 240 python bench.py > gpurun_out/b_xl.log 2>&1 || exit $?
grep streams gpurun_out/b_xl.log; grep '^{' gpurun_out/b_xl.log | cut -c1-150
