set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_$name.log 2>&1 || { tail -20 gpurun_out/bench_$name.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/bench_$name.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$name'", d["value"], d["ms_per_added_command_e2e_marginal"], d["phase_ms_per_step"]["stt"], d["llm_stats"]["gpu_wait_s"]/d["llm_stats"]["decode_steps"], d["stt_stats"]["gpu_wait_s"]/d["stt_stats"]["decode_steps"])'
}






run P1 LOQA_POOL_SKEW_PREFILL=1
run P2 LOQA_POOL_SKEW_PREFILL=2
run P3 LOQA_POOL_SKEW_PREFILL=3
run E1 LOQA_POOL_SKEW_ENCODER=1
run E2 LOQA_POOL_SKEW_ENCODER=2
run E3 LOQA_POOL_SKEW_ENCODER=3
