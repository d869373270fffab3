set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --mode hub > gpurun_out/bench_hub.log 2>&1
rc=$?; grep '^{"metric"' gpurun_out/bench_hub.log | cut -c1-600; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_hub.log; exit $rc; }
timeout -k 10 600 python -u scripts/bench_configs.py --config 2 3 > gpurun_out/configs23.log 2>&1
rc=$?; grep '^{' gpurun_out/configs23.log | cut -c1-900; [ $rc -eq 0 ] || { tail -20 gpurun_out/configs23.log; exit $rc; }
