"""Llama-3-8B decode-step wall time vs tokens per step (T = 8 per sequence x B
sequences, prompt tokens fed through the decode path), graphs captured up
front: the marginal cost of extra tokens in a memory-bound step."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd.engine.grammar import multi_command_schema  # noqa: E402
from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine  # noqa: E402
from loqa_hub_amd.engine.synthetic import make_unique  # noqa: E402
from loqa_hub_amd.llm.prompts import build_multi_command_prompt  # noqa: E402
from loqa_hub_amd.models.configs import llama_config  # noqa: E402

dev = torch.device("cuda", 0)
eng = LLMEngine(llama_config("llama3-8b"), dev, seed=0, max_seqs=16, max_seq_len=1024)
eng.warmup_graphs()
torch.cuda.synchronize()
utts = make_unique(0, [2] * 64)
out, ui = {}, 0
for B in (1, 2, 4, 8, 16):
    reqs = []
    for _ in range(B):
        r = GenRequest(eng.tok.encode(build_multi_command_prompt(utts[ui].text), bos=True),
                       multi_command_schema(2))
        ui += 1
        eng.submit(r)
        reqs.append(r)
    ts = []
    for i in range(8):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.decode_step(reqs)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts = sorted(ts[2:])
    out[f"B{B}_T{8 * B}"] = round(ts[len(ts) // 2] * 1e3, 3)
    print(out, flush=True)
    for r in reqs:
        eng.kv.pool.free_seq(r.seq_id)
print(json.dumps(out))
