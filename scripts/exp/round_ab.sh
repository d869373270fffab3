set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh || exit $?
LOQA_MPAD_PLAN=0 timeout -k 10 300 python bench.py > gpurun_out/bench_nompad.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bench_nompad.log | tail -1 | cut -c1-400; exit $rc
