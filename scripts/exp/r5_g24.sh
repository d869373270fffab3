# Whisper decoder attention split: self vs cross durations in the pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/g24prof
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g24prof -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/g24_prof.log 2>&1 || { tail -20 gpurun_out/g24_prof.log; exit 1; }
f=$(ls gpurun_out/g24prof/run_kernel_trace.csv gpurun_out/g24prof/*/run_kernel_trace.csv 2>/dev/null | head -1)
python3 - "$f" <<'PY' > gpurun_out/g24_xattn.txt
import csv, sys, statistics as st
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
att = [r for r in rows if 'attn_decode_kernel<64' in r['Kernel_Name']]
att.sort(key=lambda r: int(r['Start_Timestamp']))
# per queue: in a Whisper step, attention launches alternate self, cross
byq = {}
for r in att:
    byq.setdefault((r.get('Queue_Id'), r.get('Stream_Id')), []).append(r)
for q, lst in byq.items():
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in lst]
    wg = [int(r.get('Grid_Size_X', r.get('Grid_Size', 0)) or 0) for r in lst]
    ev, od = d[0::2], d[1::2]
    print(q, len(d), 'even median %.1f us' % st.median(ev), 'odd median %.1f us' % st.median(od),
          'grids', sorted(set(wg))[:8])
gx = {}
for r in att:
    key = (r.get('Grid_Size_X'), r.get('Grid_Size_Y'), r.get('Grid_Size_Z'))
    gx.setdefault(key, []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(gx.items(), key=lambda kv: -len(kv[1]))[:10]:
    print('grid', k, 'n', len(v), 'median %.1f us' % st.median(v))
PY
cat gpurun_out/g24_xattn.txt
rm -f "$f"
