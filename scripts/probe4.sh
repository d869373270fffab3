set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for pr in -1 0 -1 0; do
timeout -k 10 300 python bench.py --steps 4 --warmup 2 --stt-priority $pr > gpurun_out/bench_p$pr.log 2>&1 || { tail -30 gpurun_out/bench_p$pr.log; exit 1; }
echo "prio $pr: $(grep -v amdgpu.ids gpurun_out/bench_p$pr.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_added_command_e2e_marginal"], d["phase_ms_per_step"])')"
done
