set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/bench_configs.py --config 5 --tp 8 --share-gpu --compact --per-stream 1 --warmup 1 > gpurun_out/c5_tp8.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/c5_tp8.log | tail -5 | cut -c1-3000
exit $rc
