set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_$name.log 2>&1 || { tail -20 gpurun_out/bench_$name.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/bench_$name.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$name'", d["value"], d["ms_per_added_command_e2e_marginal"], d["phase_ms_per_step"]["stt"], d["llm_stats"]["gpu_wait_s"]/d["llm_stats"]["decode_steps"], d["stt_stats"]["gpu_wait_s"]/d["stt_stats"]["decode_steps"])'
}
run L1 LOQA_POOL_SKEW_LLM=1
run L2 LOQA_POOL_SKEW_LLM=2
run L3 LOQA_POOL_SKEW_LLM=3
run S1 LOQA_POOL_SKEW_STT=1
run S2 LOQA_POOL_SKEW_STT=2
run S3 LOQA_POOL_SKEW_STT=3
