set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for s in 4 5 8 12 5; do
  timeout -k 10 300 python bench.py --steps $s --warmup 2 > gpurun_out/bench_s$s.log 2>&1 || { tail -20 gpurun_out/bench_s$s.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/bench_s$s.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("steps'$s'", d["value"], d["ms_per_added_command_e2e_marginal"], d["phase_ms_per_step"])'
done
