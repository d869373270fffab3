set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
one() {
  name=$1; dir=$2
  (cd $dir && timeout -k 10 300 python bench.py --steps 4 --warmup 2) > gpurun_out/ab_$name.log 2>&1 || { tail -20 gpurun_out/ab_$name.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab_$name.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("'$name'", d["value"], d["phase_ms_per_step"]["stt"], d["llm_stats"]["gpu_wait_s"]/d["llm_stats"]["decode_steps"], d["stt_stats"]["gpu_wait_s"]/d["stt_stats"]["decode_steps"])'
}
one NEW .
timeout -k 10 900 python scripts/bench_configs.py --config 5 --per-stream 2 > gpurun_out/cfg5d.log 2>&1 || { tail -20 gpurun_out/cfg5d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cfg5d.log | tail -1 | cut -c1-500
