"""Isolated Llama-3-8B prefill of distinct ~300-token parser prompts (one
request per pass, as the serving scheduler issues them): wall time per pass.
Run under rocprofv3 --stats for the kernel breakdown."""
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
eng = LLMEngine(llama_config(os.environ.get("MODEL", "llama3-8b")), dev, seed=0, max_seqs=8,
                max_seq_len=1024)
eng.inline_prefill = 0
utts = make_unique(0, [2] * 24)
ts = []
for i, u in enumerate(utts):
    r = GenRequest(eng.tok.encode(build_multi_command_prompt(u.text), bos=True), multi_command_schema(2))
    eng.submit(r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.prefill([r])
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
    eng.kv.pool.free_seq(r.seq_id)
ts = ts[4:]
ts.sort()
print(json.dumps({"prefill_ms_median": round(ts[len(ts) // 2] * 1e3, 3), "min": round(ts[0] * 1e3, 3),
                  "tokens": eng.stats["prefill_tokens"] / len(utts)}), flush=True)
