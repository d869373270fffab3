# long steady-state run (100 timed steps) + final-tree kernel stats summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --steps 100 --warmup 5 > gpurun_out/g34_bench100.log 2>&1 || { tail -20 gpurun_out/g34_bench100.log; exit 1; }
grep -v amdgpu.ids gpurun_out/g34_bench100.log | tail -1 | cut -c1-200
rm -rf gpurun_out/g34prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g34prof -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/g34_prof.log 2>&1 || { tail -20 gpurun_out/g34_prof.log; exit 1; }
f=$(ls gpurun_out/g34prof/run_kernel_trace.csv gpurun_out/g34prof/*/run_kernel_trace.csv 2>/dev/null | head -1)
rm -f "$f"
ls gpurun_out/g34prof
