# round-end style check (GPU tests, smoke, default bench), then the config-5
# TP=8 end-to-end rehearsal (8 ranks on cuda:0); every step limited, stop at
# the first failure
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/g9_gpu_tests.log 2>&1 || { tail -30 gpurun_out/g9_gpu_tests.log; exit 1; }
tail -1 gpurun_out/g9_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/g9_smoke.log 2>&1 || { tail -20 gpurun_out/g9_smoke.log; exit 2; }
tail -1 gpurun_out/g9_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/g9_bench.log 2>&1 || { tail -20 gpurun_out/g9_bench.log; exit 3; }
grep -v amdgpu.ids gpurun_out/g9_bench.log | tail -1 | cut -c1-600
timeout -k 10 900 python -u scripts/bench_configs.py --config 5 --tp 8 --share-gpu --compact > gpurun_out/g9_c5_tp8.log 2>&1 || { tail -30 gpurun_out/g9_c5_tp8.log; exit 4; }
grep '^{' gpurun_out/g9_c5_tp8.log | tail -1 | cut -c1-900
echo alldone
