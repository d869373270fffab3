"""Llama-3-8B fused decode forward (graph-replayed, alone) vs padded rows:
what a decode step that carries prompt rows costs at Mpad 16 / 32 / 64 / 128.
B sequences x q tokens each (q <= 8, the grouped decode attention's limit),
contexts ~300 keys like the bench's prompts.

    python scripts/exp/fused_step_by_mpad.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd.engine.llm_engine import GenRequest, LLMEngine  # noqa: E402
from loqa_hub_amd.models.configs import llama_config  # noqa: E402


def main() -> int:
    dev = torch.device("cuda", 0)
    eng = LLMEngine(llama_config(os.environ.get("MODEL", "llama3-8b")), dev, seed=0, max_seqs=32,
                    max_seq_len=1024)
    out = {}
    for B, q in ((2, 8), (4, 8), (8, 8), (16, 8), (8, 4), (16, 2)):
        T = B * q
        reqs = []
        for i in range(B):
            r = GenRequest(list(range(5 + i, 305 + i)), [])
            r.seq_id = eng._next_id
            eng._next_id += 1
            eng.kv.pool.add_seq(r.seq_id, [])
            eng.kv.pool.append(r.seq_id, 300)
            reqs.append(r)
        from loqa_hub_amd import ops
        T_pad = ops.mpad_for(T)
        max_q, max_ctx, host = eng._meta(reqs, [[7] * q for _ in reqs], True, B, T_pad)
        import numpy as np
        host["mask_rows"] = np.zeros(B, np.int32)
        d = eng._to_device(host)
        meta = eng._build_meta(d, max_q, 512, True)
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            for _ in range(2):
                eng._forward_sample(meta, d["mask_rows"])
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            eng._forward_sample(meta, d["mask_rows"])
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        out[f"B{B}_q{q}_T{T}_Mpad{T_pad}"] = round(ts[len(ts) // 2], 3)
        print(json.dumps(out), flush=True)
        for r in reqs:
            eng.kv.pool.free_seq(r.seq_id)
        del g
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
