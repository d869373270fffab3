set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for u8 in 0 1; do
LOQA_WR4_U8=$u8 timeout -k 10 300 python scripts/bench_kernels.py fused > gpurun_out/kb_u$u8.log 2>&1 || { tail -30 gpurun_out/kb_u$u8.log; exit 1; }
echo "u8=$u8"; grep -v amdgpu gpurun_out/kb_u$u8.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['shape'], {k:v for k,v in d.items() if 'wr4' in k or k=='fusedS1_us'})"
done
timeout -k 10 400 python bench.py --steps 4 --warmup 2 > gpurun_out/bench1.log 2>&1 || { tail -30 gpurun_out/bench1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench1.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_added_command_e2e_marginal"], d["llm_stats"]["gpu_wait_s"]/d["llm_stats"]["decode_steps"], d["stt_stats"]["gpu_wait_s"]/d["stt_stats"]["decode_steps"])'
