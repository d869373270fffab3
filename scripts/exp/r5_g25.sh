# in-pipeline anatomy of the LLM prompt (mixed) passes: every kernel on the
# LLM queue that is not part of a decode-step graph, per pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/g25prof
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g25prof -o run -- python bench.py --steps 6 --warmup 3 > gpurun_out/g25_prof.log 2>&1 || { tail -20 gpurun_out/g25_prof.log; exit 1; }
f=$(ls gpurun_out/g25prof/run_kernel_trace.csv gpurun_out/g25prof/*/run_kernel_trace.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY' > gpurun_out/g25_mixed_anatomy.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
# mixed passes: the attn_prefill2<128 launches (32 per pass, Llama head dim 128)
pre = [r for r in rows if 'attn_prefill2_kernel<128' in r['Kernel_Name']]
npass = len(pre) / 32
q = collections.Counter((r['Queue_Id'], r.get('Stream_Id')) for r in pre).most_common(1)[0][0]
qrows = [r for r in rows if (r['Queue_Id'], r.get('Stream_Id')) == q]
agg = collections.defaultdict(float); cnt = collections.Counter()
for r in qrows:
    n = r['Kernel_Name']
    if ('skinny' in n and 'gemm_sk' not in n) or 'attn_decode' in n or 'argmax' in n:
        continue   # decode-step graphs share the queue (and the split attention's decode launches)
    agg[n] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    cnt[n] += 1
print(f"{npass:.1f} prompt passes (queue {q}); per pass:")
tot = 0
for n, t in sorted(agg.items(), key=lambda kv: -kv[1])[:16]:
    tot += t / npass
    print(f"  {t / npass:8.1f} us  {cnt[n] / npass:6.1f} calls  {n[:100]}")
print(f"  total of the listed kernels {tot:.0f} us per pass")
PY
cat gpurun_out/g25_mixed_anatomy.txt
rm -f "$f"
