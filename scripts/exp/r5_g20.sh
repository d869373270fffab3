# LDS conv with register-staged, prefetched chunks: numerics + VITS timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "conv or vits or tts" > gpurun_out/g20_tests.txt 2>&1 || exit 11
tail -2 gpurun_out/g20_tests.txt
for n in 1 2 8; do
  timeout -k 10 200 python -u scripts/exp/vits_prof.py --iters 10 --phrases $n > gpurun_out/g20_vits_p$n.json 2>&1 || exit 12
  grep '^{' gpurun_out/g20_vits_p$n.json | cut -c1-120
done
echo done
