set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
for i in 1 2; do
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/bench$i.log 2>&1 || { tail -30 gpurun_out/bench$i.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench$i.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_added_command_e2e_marginal"], d["phase_ms_per_step"]["stt"], d["llm_stats"]["gpu_wait_s"]/d["llm_stats"]["decode_steps"], d["stt_stats"]["gpu_wait_s"]/d["stt_stats"]["decode_steps"], {k:v for k,v in d["fused_gemm_tuning"].items() if "1280" in k})'
done
