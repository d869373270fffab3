set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_long_form.py > gpurun_out/g1_lf.txt 2>&1 || exit 11
timeout -k 10 240 python -u scripts/frontend_bench.py --relays 64 --workers 8 --seconds 30 --client-procs 4 > gpurun_out/g1_fe64.json 2> gpurun_out/g1_fe64.err || exit 12
timeout -k 10 240 python -u scripts/frontend_bench.py --relays 64 --workers 8 --seconds 30 --client-procs 4 --shm-slots 0 > gpurun_out/g1_fe64_noshm.json 2> gpurun_out/g1_fe64_noshm.err || exit 13
LOQA_PCM_STREAM_IN=1 timeout -k 10 400 python -u bench.py --mode hub --paced --steps 6 --warmup 2 > gpurun_out/g1_paced_on.json 2> gpurun_out/g1_paced_on.err || exit 14
LOQA_PCM_STREAM_IN=0 timeout -k 10 400 python -u bench.py --mode hub --paced --steps 6 --warmup 2 > gpurun_out/g1_paced_off.json 2> gpurun_out/g1_paced_off.err || exit 15
echo done
