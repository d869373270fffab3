set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/finalprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/finalprof -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/final_prof.log 2>&1 || { tail -20 gpurun_out/final_prof.log; exit 1; }
f=$(ls gpurun_out/finalprof/run_kernel_trace.csv gpurun_out/finalprof/*/run_kernel_trace.csv 2>/dev/null | head -1)
python scripts/decode_steps.py "$f" llm > gpurun_out/final_anatomy.txt 2>&1
python scripts/decode_steps.py "$f" stt > gpurun_out/final_anatomy_stt.txt 2>&1
head -16 gpurun_out/final_anatomy.txt; head -12 gpurun_out/final_anatomy_stt.txt
rm -f "$f"
