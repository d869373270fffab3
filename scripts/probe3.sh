set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof.log 2>&1
rc=$?
echo "profile rc=$rc"
grep -v amdgpu.ids gpurun_out/prof.log | tail -1 | cut -c1-300
exit $rc
