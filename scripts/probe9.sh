set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/bench_$name.log 2>&1 || { tail -20 gpurun_out/bench_$name.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/bench_$name.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$name'", d["value"], d["ms_per_added_command_e2e_marginal"], d["phase_ms_per_step"]["stt"], d["llm_stats"]["gpu_wait_s"]/d["llm_stats"]["decode_steps"], d["stt_stats"]["gpu_wait_s"]/d["stt_stats"]["decode_steps"])'
}
run GU_S2 "LOQA_FSPLIT_OVERRIDE=silu:28672x4096:M16=2,2,1;silu:28672x4096:M32=2,2,1"
run GU_S2_UNCAP LOQA_MAX_DECODE_WGS=100000 "LOQA_FSPLIT_OVERRIDE=silu:28672x4096:M16=2,2,1;silu:28672x4096:M32=2,2,1;rope:6144x4096:M16=1,2,1"
run BASE X=1
