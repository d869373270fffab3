# Infinity Cache weight prefetch: equivalence test, config-5 rank step, 8B A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_engine_gpu.py -k "l3_prefetch or pipelined" > gpurun_out/g9_tests.txt 2>&1 || exit 11
for v in "base|LOQA_L3_PREFETCH=0" "pf128|LOQA_L3_PREFETCH=1 LOQA_L3_PREFETCH_WGS=128" "pf256|LOQA_L3_PREFETCH=1 LOQA_L3_PREFETCH_WGS=256" "pf64|LOQA_L3_PREFETCH=1 LOQA_L3_PREFETCH_WGS=64"; do
  label="${v%%|*}"; envs="${v#*|}"
  env $envs timeout -k 10 400 python -u scripts/config5_projection.py --iters 30 --prefill-rows 0 > gpurun_out/g9_c5_${label}.json 2> gpurun_out/g9_c5_${label}.err || exit 12
  echo "$label $(cut -c1-330 gpurun_out/g9_c5_${label}.json)"
done
AB="p0|LOQA_L3_PREFETCH=0;p1|LOQA_L3_PREFETCH=1" bash scripts/exp/bench_ab.sh > gpurun_out/g9_ab.txt 2>&1 || exit 13
cat gpurun_out/g9_ab.txt
echo done
