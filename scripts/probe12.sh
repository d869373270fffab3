set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/cliffprof
LOQA_STT_MAX_WGS=128 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cliffprof -o run -- python bench.py --steps 3 --warmup 2 > gpurun_out/cliff_prof.log 2>&1 || { tail -20 gpurun_out/cliff_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cliff_prof.log | grep '^{' | cut -c1-200
f=$(ls gpurun_out/cliffprof/run_kernel_trace.csv gpurun_out/cliffprof/*/run_kernel_trace.csv 2>/dev/null | head -1)
python scripts/decode_steps.py "$f" llm > gpurun_out/cliff_anatomy.txt 2>&1
python scripts/decode_steps.py "$f" stt >> gpurun_out/cliff_anatomy.txt 2>&1
python - "$f" <<'PY' >> gpurun_out/cliff_anatomy.txt
import csv, sys, statistics as st
rows=[(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50], r.get("Queue_Id"), r.get("Stream_Id")) for r in csv.DictReader(open(sys.argv[1]))]
rows.sort()
# concurrency: fraction of time with >=2 kernels running
ev=[]
for a,b,*_ in rows: ev += [(a,1),(b,-1)]
ev.sort(); cur=0; last=ev[0][0]; acc={}
for t,d in ev:
    acc[cur]=acc.get(cur,0)+(t-last); cur+=d; last=t
tot=sum(acc.values())
print("concurrency histogram:", {k: round(v/tot,3) for k,v in sorted(acc.items())})
qs={}
for r in rows: qs[(r[3],r[4])]=qs.get((r[3],r[4]),0)+1
print("dispatches per (queue, stream):", sorted(qs.items(), key=lambda x:-x[1])[:12])
PY
cat gpurun_out/cliff_anatomy.txt
rm -f "$f"
