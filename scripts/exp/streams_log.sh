set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp LOQA_LOG_STREAMS=1
(cd _old && timeout -k 10 300 python bench.py --steps 2 --warmup 1 > ../gpurun_out/streams_old.log 2>&1) || exit $?
grep "streams\]\|^{" gpurun_out/streams_old.log | cut -c1-160
timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/streams_new.log 2>&1 || exit $?
grep "streams\]\|^{" gpurun_out/streams_new.log | cut -c1-160
