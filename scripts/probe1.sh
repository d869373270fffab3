set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1; do
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/bench$i.log 2>&1 || { tail -30 gpurun_out/bench$i.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench$i.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_added_command_e2e_marginal"], d["phase_ms_per_step"], d["llm_stats"], d["stt_stats"])'
done
