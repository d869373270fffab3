set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "prefill_gemm2" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pg2_test.log 2>&1
rc=$?; tail -3 gpurun_out/pg2_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/exp/prefill_gemm2_bench.py > gpurun_out/pg3_bench.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/pg3_bench.log | python3 -c "
import json,sys
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    us={k:v for k,v in d.items() if k.endswith('_us')}
    print(d['gemm'], sorted(us.items(), key=lambda kv: kv[1])[:6])
"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode hub --window-ms 20 > gpurun_out/bench_hub20.log 2>&1
rc=$?; grep '^{"metric"' gpurun_out/bench_hub20.log | cut -c1-300; exit $rc
