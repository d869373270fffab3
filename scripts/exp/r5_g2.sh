set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/config5_projection.py --iters 30 > gpurun_out/g2_c5proj.json 2> gpurun_out/g2_c5proj.err || exit 11
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/g2_c5prof -o c5 -- python -u scripts/config5_projection.py --iters 10 --layers 8 > gpurun_out/g2_c5prof.log 2>&1 || exit 12
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/g2_tp.txt 2>&1 || exit 13
echo done
