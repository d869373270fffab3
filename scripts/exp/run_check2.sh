set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -k splitk -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sk.log 2>&1
rc=$?; tail -2 gpurun_out/t_sk.log; [ $rc = 0 ] || exit $rc
LOQA_PREFILL_O_SPLITS=0 timeout -k 10 200 python scripts/exp/prefill_prof.py > gpurun_out/pf_o0.log 2>&1 || exit $?
timeout -k 10 200 python scripts/exp/prefill_prof.py > gpurun_out/pf_o4.log 2>&1 || exit $?
tail -1 gpurun_out/pf_o0.log; tail -1 gpurun_out/pf_o4.log
