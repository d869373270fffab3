"""Isolated Llama-3-8B prompt-pass time vs rows per pass (the hand-written
GEMM path, graph-free, as the scheduler issues it): what a chunked prompt pass
of M rows costs next to a full ~300-row pass and a 16-row decode step.

    python scripts/exp/prefill_m_sweep.py [--ms 32,64,128,192,256,320]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd.engine.grammar import multi_command_schema  # noqa: E402
from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine  # noqa: E402
from loqa_hub_amd.models.configs import llama_config  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="32,64,96,128,160,192,256,320")
    ap.add_argument("--reps", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = LLMEngine(llama_config("llama3-8b"), dev, seed=0, max_seqs=8, max_seq_len=1024)
    g = torch.Generator().manual_seed(0)
    out = {}
    for M in (int(v) for v in a.ms.split(",")):
        ts = []
        for i in range(a.reps):
            toks = torch.randint(3, 30000, (M,), generator=g).tolist()
            r = GenRequest(toks, multi_command_schema(1))
            eng.submit(r)
            max_q, max_ctx, host = eng._meta([r], [r.feed], decode=False)
            dev_m = eng._to_device(host)
            meta = eng._build_meta(dev_m, max_q, max_ctx, False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hid = eng.model.forward(meta, eng.kv.k, eng.kv.v, eng.attn_ws)
            eng.model.logits(hid)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            eng.kv.pool.free_seq(r.seq_id)
        ts = sorted(ts[2:])
        out[M] = round(ts[len(ts) // 2] * 1e3, 3)
        print(json.dumps({"M": M, "ms": out[M]}), flush=True)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
