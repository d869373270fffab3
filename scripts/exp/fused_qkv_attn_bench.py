"""qkv GEMM + decode attention: two launches vs the fused launch
(skinny_fused(attn=), gemm_skinny.hip ATTD), graph-replayed, per layer, on
the pipeline's decode shapes (Llama-3-8B and Whisper large-v3 decoder).
Each layer of a step reads its own weight copy (cold weights, as in a step).

    python scripts/exp/fused_qkv_attn_bench.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402
from tests.test_fused_qkv_attn import SHAPES, _case  # noqa: E402

LAYERS = 16


def bench(shape, Mpad, max_q, fuse, rt, wr, S, ctx_scale=1.0):
    c = _case(shape, Mpad, max_q, seed=1)
    dev = c["x"].device
    H, Hkv, D = c["H"], c["Hkv"], c["D"]
    lins = [c["lin"]]
    for _ in range(LAYERS - 1):
        import copy
        l2 = copy.copy(c["lin"])
        l2.wp = c["lin"].wp.clone()
        lins.append(l2)
    ws = ops.AttnWorkspace(dev, 64, H, D, 64)
    scr = ops.FusedScratch(dev)
    scr.seed_stats(c["x"])
    q = torch.empty(Mpad, H * D, dtype=torch.bfloat16, device=dev)
    out = torch.empty(Mpad, H * D, dtype=torch.bfloat16, device=dev)
    ns, sk = ops.decode_attn_splits(c["max_ctx"], c["B"] * Hkv, 128)
    ops.FUSE_QKV_ATTN = fuse

    def step():
        for lin in lins:
            ops.skinny_fused(c["x"], lin, "rope", scr, splits=S, rt=rt, wr=wr, xl=0, eps=1e-5,
                             rowsq_tiles=1, positions=c["pos"], cos_sin=c["cs"], q_out=q,
                             k_cache=c["kc"], v_cache=c["vc"], slots=c["slots"], n_heads=H,
                             n_kv=Hkv, head_dim=D,
                             attn=dict(cu_q=c["cu_q"], ctx_lens=c["ctx"], block_tables=c["bt"],
                                       max_q=max_q, split_keys=sk, num_splits=ns, workspace=ws,
                                       out=out))
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000 / LAYERS)
    ts.sort()
    assert int(ws.sync.abs().sum()) == 0, ws.sync[:80].tolist()
    return round(ts[len(ts) // 2], 2), c["B"], c["max_ctx"]


def bench_x(Mpad, max_q, fuse, rt, wr, S):
    from tests.test_fused_qkv_attn import _xcase
    c = _xcase(Mpad, max_q, seed=1)
    dev = c["x"].device
    ws = ops.AttnWorkspace(dev, 64, c["H"], c["D"], 64)
    scr = ops.FusedScratch(dev)
    scr.seed_stats(c["x"])
    out = torch.empty(Mpad, c["K"], dtype=torch.bfloat16, device=dev)
    ao = torch.empty(Mpad, c["K"], dtype=torch.bfloat16, device=dev)
    lins = [c["lin"]]
    import copy
    for _ in range(LAYERS - 1):
        l2 = copy.copy(c["lin"])
        l2.wp = c["lin"].wp.clone()
        lins.append(l2)
    ops.FUSE_QKV_ATTN = fuse

    def step():
        for lin in lins:
            ops.skinny_fused(c["x"], lin, "act", scr, splits=S, rt=rt, wr=wr, xl=0, eps=1e-5,
                             rowsq_tiles=1, out=out, n_heads=c["H"], n_kv=c["H"], head_dim=c["D"],
                             attn=dict(cu_q=c["cu_q"], ctx_lens=c["lens"], kv_start=c["starts"],
                                       k=c["kv"], v=c["kv"][:, c["K"]:], max_q=max_q,
                                       split_keys=512, num_splits=3, workspace=ws, out=ao))
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000 / LAYERS)
    ts.sort()
    assert int(ws.sync.abs().sum()) == 0, ws.sync[:80].tolist()
    return round(ts[len(ts) // 2], 2), c["B"]


def main():
    for Mpad, max_q in ((16, 1), (16, 4), (32, 1)):
        for rt, wr, S in ((1, 1, 1), (2, 1, 1)):
            r = {"shape": "whisper_cross", "Mpad": Mpad, "max_q": max_q, "rt": rt, "wr": wr, "S": S}
            r["two_launch_us"], r["B"] = bench_x(Mpad, max_q, False, rt, wr, S)
            r["fused_us"] = bench_x(Mpad, max_q, True, rt, wr, S)[0]
            print(json.dumps(r), flush=True)
    main_self()


def main_self():
    res = []
    for shape, Mpad, max_q in (("llama", 16, 1), ("llama", 32, 1), ("llama", 16, 4),
                               ("whisper", 16, 1), ("whisper", 32, 1), ("whisper", 64, 4)):
        N = (SHAPES[shape][0] + 2 * SHAPES[shape][1]) * SHAPES[shape][2]
        for rt, wr, S in ((2, 1, 1), (1, 1, 1), (2, 4, 1), (1, 4, 1), (2, 1, 2)):
            if (N // (16 * rt * wr)) * S > 256 or (wr == 4 and N % (64 * rt)):
                continue
            r = {"shape": shape, "Mpad": Mpad, "max_q": max_q, "rt": rt, "wr": wr, "S": S}
            r["two_launch_us"], r["B"], r["max_ctx"] = bench(shape, Mpad, max_q, False, rt, wr, S)
            r["fused_us"] = bench(shape, Mpad, max_q, True, rt, wr, S)[0]
            res.append(r)
            print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
