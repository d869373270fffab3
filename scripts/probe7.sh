set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cap in 128 192 384; do
LOQA_MAX_DECODE_WGS=$cap timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/bench_c$cap.log 2>&1 || { tail -20 gpurun_out/bench_c$cap.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_c$cap.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("cap '$cap'", d["value"], d["ms_per_added_command_e2e_marginal"], d["llm_stats"]["gpu_wait_s"]/d["llm_stats"]["decode_steps"], d["stt_stats"]["gpu_wait_s"]/d["stt_stats"]["decode_steps"])'
done
