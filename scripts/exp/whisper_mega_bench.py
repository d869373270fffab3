"""Whisper-large-v3 decoder step, graph-replayed device time: the persistent
one-launch step (decode_step_mega) vs the fused 8-launches-per-layer step
(decode_step_fused), at B sequences x 1 token with ~24 tokens of context.
Optional LOAD=1: a concurrent HBM-streaming load on a second stream (the
LLM decode's weight reads) while timing."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest  # noqa: E402
from loqa_hub_amd.engine.synthetic import make_batch  # noqa: E402
from loqa_hub_amd.models.configs import whisper_config  # noqa: E402
from loqa_hub_amd.models.whisper import decode_step_fused, decode_step_mega  # noqa: E402

dev = torch.device("cuda", 0)
os.environ["LOQA_STT_MEGA"] = "1"
cfg = whisper_config(os.environ.get("MODEL", "whisper-large-v3"))
eng = STTEngine(cfg, dev, seed=0, max_batch=8, use_graphs=False)
grids = [int(g) for g in os.environ.get("GRIDS", "256").split(",")]
out = []
for B in [int(b) for b in os.environ.get("BS", "1,4,8").split(",")]:
    utts = make_batch(0, B, [2])
    reqs = [STTRequest(u.pcm) for u in utts]
    audio, _ = eng.upload(reqs)
    eng.cross_kv(eng.model.encode(audio))
    for i, r in enumerate(reqs):
        r.seq_id = eng._next
        r.slot = i
        eng._next += 1
        eng.kv.pool.add_seq(r.seq_id, [])
        r.feed = list(range(100, 124))          # 24 tokens of context
    for r in reqs:                              # allocate the context positions
        eng._host_meta([r], 1, 32)
        r.feed = [7]
    max_q, host = eng._host_meta(reqs, B, 16)
    d = eng._dev(host)
    res = {"B": B}
    variants = [("fused", None)] + [(f"mega{g}", g) for g in grids]
    for name, g in variants:
        def step():
            if g is None:
                return decode_step_fused(eng.model, d["tokens"], d["positions"], d["slots"], d["cu_q"],
                                         d["ctx_lens"], d["block_tables"], 1, eng.kv.k, eng.kv.v, eng.xkv,
                                         d["enc_starts"], d["enc_lens"], d["logit_idx"], eng.ws,
                                         eng.scratch, 1)
            eng.mega.grid = g
            return decode_step_mega(eng.model, d["tokens"], d["positions"], d["slots"], d["cu_q"],
                                    d["ctx_lens"], d["block_tables"], d["enc_starts"], d["enc_lens"],
                                    d["logit_idx"], eng.mega)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream(dev).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        for _ in range(3):
            graph.replay()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        n = 30
        ev[0].record()
        for _ in range(n):
            graph.replay()
        ev[1].record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(ev[0].elapsed_time(ev[1]) * 1e3 / n, 1)
        if g is not None:
            res[name + "_err"] = eng.mega.error()
    print(json.dumps(res), flush=True)
    for r in reqs:
        eng.kv.pool.free_seq(r.seq_id)

# per-item timeline of one step (s_memrealtime, 100 MHz): B = 4
if os.environ.get("TIMELINE", "1") == "1":
    import numpy as np
    B = 4
    utts = make_batch(0, B, [2])
    reqs = [STTRequest(u.pcm) for u in utts]
    audio, _ = eng.upload(reqs)
    eng.cross_kv(eng.model.encode(audio))
    for i, r in enumerate(reqs):
        r.seq_id = eng._next
        r.slot = i
        eng._next += 1
        eng.kv.pool.add_seq(r.seq_id, [])
        r.feed = list(range(100, 124))
    for r in reqs:
        eng._host_meta([r], 1, 32)
        r.feed = [7]
    max_q, host = eng._host_meta(reqs, B, 16)
    d = eng._dev(host)
    m = eng.mega
    m.grid = grids[0]
    H, dd = m.H, m.d
    n = [3 * dd // 16, B * H, dd // 16, dd // 16, B * H * m.nsplit, dd // 16, m.F // 16, dd // 16]
    C = sum(n)
    m.dbg = torch.zeros(C * m.L * 5, dtype=torch.int64, device=dev)
    for _ in range(3):
        decode_step_mega(eng.model, d["tokens"], d["positions"], d["slots"], d["cu_q"], d["ctx_lens"],
                         d["block_tables"], d["enc_starts"], d["enc_lens"], d["logit_idx"], m)
    torch.cuda.synchronize()
    ts = m.dbg.view(m.L, C, 5).cpu().numpy().astype(np.float64) * 10.0 / 1e3   # -> us
    m.dbg = None
    off = np.cumsum([0] + n)
    t_first = ts[:, :, 0].min()
    print(json.dumps({"step_us": round(float(ts[:, :, 4].max() - t_first), 1)}), flush=True)
    for l in (0, 5, 6):
        base = ts[l, :, 1].min()
        rows = []
        for ph in range(8):
            x = ts[l, off[ph]:off[ph + 1]]
            rows.append({"ph": ph, "n": int(n[ph]), "t1_min": round(float(x[:, 1].min() - base), 1),
                         "t1_max": round(float(x[:, 1].max() - base), 1),
                         "t3_max": round(float(x[:, 3].max() - base), 1),
                         "t4_max": round(float(x[:, 4].max() - base), 1),
                         "stage_med": round(float(np.median(x[:, 2] - x[:, 1])), 2),
                         "work_med": round(float(np.median(x[:, 3] - x[:, 2])), 2),
                         "signal_med": round(float(np.median(x[:, 4] - x[:, 3])), 2)})
        print(json.dumps({"layer": l, "phases": rows}), flush=True)
