"""Where the time between two LLM decode steps goes (Llama-3-8B, 8 sequences,
no concurrent STT): back-to-back graph replays (GPU only) vs replay + result
read-back per step vs the engine's full decode_step (grammar advance, step
metadata, H2D copy, replay, read-back)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd.engine.grammar import multi_command_schema  # noqa: E402
from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine  # noqa: E402
from loqa_hub_amd.llm.prompts import build_multi_command_prompt  # noqa: E402
from loqa_hub_amd.models.configs import llama_config  # noqa: E402

dev = torch.device("cuda", 0)
model = os.environ.get("MODEL", "llama3-8b")
B = int(os.environ.get("B", "8"))
eng = LLMEngine(llama_config(model), dev, seed=0, max_seqs=B, max_seq_len=1024)
eng.inline_prefill = 0
eng.warmup_graphs()
torch.cuda.synchronize()
prompt = eng.tok.encode(build_multi_command_prompt("turn on the kitchen lights and play music"), bos=True)
reqs = [GenRequest(list(prompt), multi_command_schema(4, min_response_tokens=8)) for _ in range(B)]
for r in reqs:
    eng.submit(r)
eng.prefill(reqs)
torch.cuda.synchronize()
live = [r for r in reqs if not r.done]
out = {}
# optional: a background thread running pure-Python work (GIL contention)
if os.environ.get("GIL_HOG"):
    import threading
    stop = [False]

    def hog():
        x = 0
        while not stop[0]:
            for i in range(2000):
                x += i * i
            time.sleep(float(os.environ["GIL_HOG"]))
    th = threading.Thread(target=hog, daemon=True)
    th.start()
# full engine steps
ts = []
per_t = {}
for _ in range(60):
    T = sum(min(len(r.feed), eng.max_decode_q) for r in live)
    t0 = time.perf_counter()
    eng.decode_step(live)
    ts.append(time.perf_counter() - t0)
    per_t.setdefault(16 if T <= 16 else 32 if T <= 32 else 64, []).append(ts[-1] * 1e3)
    live = [r for r in live if not r.done]
out["step_ms_by_T"] = {k: [round(min(v), 2), round(sorted(v)[len(v) // 2], 2), len(v)] for k, v in per_t.items()}
ts.sort()
out["decode_step_ms_median"] = round(ts[len(ts) // 2] * 1e3, 3)
out["decode_step_ms_p90"] = round(ts[int(len(ts) * 0.9)] * 1e3, 3)
for key, gg in sorted(eng._graphs.items()):
    if key[0] != B or key[2] != 512:
        continue
    for _ in range(3):
        gg["graph"].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        gg["graph"].replay()
    torch.cuda.synchronize()
    out[f"replay_T{key[1]}_ms"] = round((time.perf_counter() - t0) / 20 * 1e3, 3)
g = next(v for k, v in eng._graphs.items() if k[0] == B and k[1] == 16)
# back-to-back replays (GPU time per step, no host turnaround)
for _ in range(3):
    g["graph"].replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(30):
    g["graph"].replay()
torch.cuda.synchronize()
out["replay_back_to_back_ms"] = round((time.perf_counter() - t0) / 30 * 1e3, 3)
# replay + read-back each step
ts = []
for _ in range(30):
    t0 = time.perf_counter()
    g["graph"].replay()
    g["out"][:B].cpu()
    ts.append(time.perf_counter() - t0)
ts.sort()
out["replay_plus_readback_ms"] = round(ts[len(ts) // 2] * 1e3, 3)
# replay + H2D metadata copies + read-back
ts = []
for _ in range(30):
    t0 = time.perf_counter()
    g["d32"].copy_(g["h32"], non_blocking=True)
    g["d64"].copy_(g["h64"], non_blocking=True)
    g["graph"].replay()
    g["out"][:B].cpu()
    ts.append(time.perf_counter() - t0)
ts.sort()
out["h2d_replay_readback_ms"] = round(ts[len(ts) // 2] * 1e3, 3)
# CPU cost of the replay call itself
torch.cuda.synchronize()
t0 = time.perf_counter()
g["graph"].replay()
out["replay_call_cpu_us"] = round((time.perf_counter() - t0) * 1e6, 1)
torch.cuda.synchronize()
out["stats"] = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in eng.stats.items()}
print(json.dumps(out), flush=True)
