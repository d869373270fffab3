set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "hub_server" > gpurun_out/r4_hub_gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r4_hub_gpu_tests.log; exit 1; }
tail -5 gpurun_out/r4_hub_gpu_tests.log
timeout -k 10 420 python bench.py --mode hub --gpus 1 --tts --steps 8 --warmup 2 --window-ms 20 > gpurun_out/r4_hub_tts_n1.json 2> gpurun_out/r4_hub_tts_n1.err || { echo BENCHFAIL; tail -30 gpurun_out/r4_hub_tts_n1.err; exit 1; }
tail -c 600 gpurun_out/r4_hub_tts_n1.json
