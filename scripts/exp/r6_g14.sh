# the driver's multi-rank bench launch, rehearsed with 2 ranks sharing cuda:0
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
LOQA_DIST_SHARE_GPU=1 LOQA_NO_TUNE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 4 --warmup 1 > gpurun_out/g14_dp2.log 2>&1 || { tail -40 gpurun_out/g14_dp2.log; exit 5; }
grep '^{' gpurun_out/g14_dp2.log | tail -1 | cut -c1-900
echo alldone
