set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
LOQA_PREFILL_DOWN_SPLITS=0 timeout -k 10 200 python scripts/exp/prefill_prof.py > gpurun_out/pf_s0.log 2>&1 || exit $?
timeout -k 10 200 python scripts/exp/prefill_prof.py > gpurun_out/pf_s8.log 2>&1 || exit $?
tail -1 gpurun_out/pf_s0.log; tail -1 gpurun_out/pf_s8.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b_sk.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/b_sk.log | tail -1 | cut -c1-1200
