# which hardware queue each serving engine's kernels use (rocprofv3 kernel
# trace Queue_Id / Stream_Id per kernel family) in the default bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/g11_prof
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g11_prof -o b -- python bench.py --steps 4 --warmup 2 --window-steps 0 > gpurun_out/g11_bench.log 2>&1 || { tail -20 gpurun_out/g11_bench.log; exit 3; }
f=$(ls gpurun_out/g11_prof/b_kernel_trace.csv gpurun_out/g11_prof/*/b_kernel_trace.csv 2>/dev/null | head -1)
python - "$f" <<'PY' > gpurun_out/g11_queues.txt
import csv, re, sys, collections
fam = [("stt_dec", re.compile(r"skinny_fused_kernel<\d, \d, 2, |attn_decode_kernel<64|skinny_gemm_kernel<2, 1, 2>")),
       ("llm_dec", re.compile(r"skinny_fused_kernel<\d, \d, 4, |attn_decode_kernel<128|skinny_gemm_kernel<2, 1, 4>")),
       ("prefill", re.compile(r"gemm_ws|gemm_sk|attn_prefill2_kernel<128")),
       ("encoder", re.compile(r"attn_prefill2_kernel<64|layernorm_kernel|log_mel|conv")),
       ("step_io", re.compile(r"step_fetch|step_publish|masked_argmax|argmax_unpack|embed_stats"))]
rows = list(csv.DictReader(open(sys.argv[1])))
print("columns:", [k for k in rows[0].keys()])
cnt = collections.Counter()
for r in rows:
    for n, p in fam:
        if p.search(r["Kernel_Name"]):
            cnt[(n, r.get("Queue_Id", "?"), r.get("Stream_Id", "?"))] += 1
            break
for k, v in sorted(cnt.items()):
    print(k, v)
PY
cat gpurun_out/g11_queues.txt
rm -rf gpurun_out/g11_prof
echo queuesdone
# served-hub soak: 150 timed steps (1200 utterances) on the default bench, with
# the process's peak GPU memory and the hub's counters
timeout -k 10 600 python bench.py --steps 150 --warmup 5 --window-steps 0 > gpurun_out/g11_soak.log 2>&1 || { tail -20 gpurun_out/g11_soak.log; exit 4; }
python - gpurun_out/g11_soak.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
h = d["hub"]
print("soak", d["value"], "utt/s", d["steps"], "steps", "ms/added", d["ms_per_added_command_e2e_marginal"],
      "events", h["voice_events"], "timed", h["timed_utterances"], "p50", h["latency_ms_p50"], "p90", h["latency_ms_p90"],
      "match", d["command_count_match_rate"], "ok", d["queue_success_rate"], "errors", h["processor"]["errors"])
PY
echo soakdone
