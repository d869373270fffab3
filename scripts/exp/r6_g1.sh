# round 6 first box: default (served hub) bench vs closed loop, config-5 rank
# step + its anatomy, 8B decode anatomy, then the kernel / engine GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/g1_bench_hub.log 2>&1 || { tail -20 gpurun_out/g1_bench_hub.log; exit 11; }
grep '^{' gpurun_out/g1_bench_hub.log | cut -c1-420
timeout -k 10 400 python bench.py --mode closed > gpurun_out/g1_bench_closed.log 2>&1 || { tail -20 gpurun_out/g1_bench_closed.log; exit 12; }
grep '^{' gpurun_out/g1_bench_closed.log | cut -c1-300
timeout -k 10 400 python -u scripts/config5_projection.py --iters 30 > gpurun_out/g1_c5proj.json 2> gpurun_out/g1_c5proj.err || { tail -20 gpurun_out/g1_c5proj.err; exit 13; }
cut -c1-600 gpurun_out/g1_c5proj.json
rm -rf gpurun_out/g1_c5prof
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g1_c5prof -o c5 -- python -u scripts/config5_projection.py --iters 10 --prefill-rows 0 > gpurun_out/g1_c5prof.log 2>&1 || { tail -20 gpurun_out/g1_c5prof.log; exit 14; }
f=$(ls gpurun_out/g1_c5prof/c5_kernel_trace.csv gpurun_out/g1_c5prof/*/c5_kernel_trace.csv 2>/dev/null | head -1)
python scripts/decode_steps.py "$f" tp > gpurun_out/g1_c5_anatomy.txt 2>&1; cat gpurun_out/g1_c5_anatomy.txt
gzip -c "$f" > gpurun_out/g1_c5_trace.csv.gz; rm -rf gpurun_out/g1_c5prof
rm -rf gpurun_out/g1_prof
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g1_prof -o b -- python bench.py --mode closed --steps 8 --warmup 3 > gpurun_out/g1_prof.log 2>&1 || { tail -20 gpurun_out/g1_prof.log; exit 15; }
f=$(ls gpurun_out/g1_prof/b_kernel_trace.csv gpurun_out/g1_prof/*/b_kernel_trace.csv 2>/dev/null | head -1)
python scripts/decode_steps.py "$f" llm > gpurun_out/g1_llm_anatomy.txt 2>&1; cat gpurun_out/g1_llm_anatomy.txt
python scripts/decode_steps.py "$f" stt > gpurun_out/g1_stt_anatomy.txt 2>&1; cat gpurun_out/g1_stt_anatomy.txt
gzip -c "$f" > gpurun_out/g1_bench_trace.csv.gz; rm -rf gpurun_out/g1_prof
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_tp_gpu.py tests/test_engine_gpu.py -m gpu > gpurun_out/g1_tests.txt 2>&1 || { tail -30 gpurun_out/g1_tests.txt; exit 16; }
tail -3 gpurun_out/g1_tests.txt
echo done
