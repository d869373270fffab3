# served hub (gRPC relays -> front end -> DP GPU worker) with the 300 ms
# arbitration window vs the single-relay bypass (every relay its own group)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --mode hub --served-dp --steps 8 --warmup 2 > gpurun_out/g13_hub_window.log 2>&1 || exit 11
grep '^{' gpurun_out/g13_hub_window.log | tail -1 | cut -c1-300
timeout -k 10 500 python -u bench.py --mode hub --served-dp --steps 8 --warmup 2 --bypass > gpurun_out/g13_hub_bypass.log 2>&1 || exit 12
grep '^{' gpurun_out/g13_hub_bypass.log | tail -1 | cut -c1-300
echo done
