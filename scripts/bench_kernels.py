#!/usr/bin/env python3
"""Kernel micro-benchmarks on the GPU (HIP-event timing, median of N reps).

Decode-step shapes of Llama-3-8B (M = 16/32 tokens): our skinny GEMM at each
split-K vs hipBLASLt (torch.nn.functional.linear); decode attention; slab ops.
Prints one JSON line per measurement (also written to gpurun_out/kbench.jsonl).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda")
out_path = "gpurun_out/kbench.jsonl"
os.makedirs("gpurun_out", exist_ok=True)
fout = open(out_path, "a")


def timeit(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def gtime(fn, inner=20, reps=10):
    """Per-call time of ``fn`` replayed from a captured HIP graph of ``inner``
    back-to-back calls (in-graph cost: no host launch overhead)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / inner)
    ts.sort()
    return ts[len(ts) // 2]


def emit(**kw):
    print(json.dumps(kw), flush=True)
    fout.write(json.dumps(kw) + "\n")


def gemm_bench():
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    for M in (16, 32, 64):
        for name, (N, K) in shapes.items():
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            wp = ops.shuffle_weight(w)
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            gb = N * K * 2 / 1e9
            t_blas = timeit(lambda: torch.nn.functional.linear(x, w))
            res = {"kernel": "gemm", "shape": name, "M": M, "N": N, "K": K,
                   "hipblaslt_us": round(t_blas, 2), "hipblaslt_TBps": round(gb / t_blas * 1e3, 2)}
            for S in (1, 2, 4, 8):
                if K % (S * 128):
                    continue
                t = timeit(lambda: ops.skinny_gemm(x, wp, S))
                res[f"skinny_S{S}_us"] = round(t, 2)
                res[f"skinny_S{S}_TBps"] = round(gb / t * 1e3, 2)
            res["auto_S"] = ops.choose_splits(N, K, M)
            emit(**res)
            del w, wp


def attn_bench():
    H, Hkv, D, blk = 32, 8, 128, 16
    for B, ctx in ((8, 450), (8, 900), (32, 450)):
        nblk = B * ((ctx + blk - 1) // blk)
        kc = torch.randn(nblk, Hkv, blk, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(nblk, dtype=torch.int32, device=dev).view(B, -1)
        q = torch.randn(B, H * D, device=dev, dtype=torch.bfloat16)
        cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
        cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        ws = ops.AttnWorkspace(dev, 256, H, D, 32)
        gb = 2 * B * ctx * Hkv * D * 2 / 1e9
        for sk in (64, 128, 256):
            ns = (ctx + sk - 1) // sk
            t = timeit(lambda: ops.attention(q, kc, vc, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=True,
                                             max_q=1, ctx_lens=cl, block_tables=bt, grouped=True,
                                             split_keys=sk, num_splits=ns, workspace=ws))
            emit(kernel="decode_attn", B=B, ctx=ctx, split_keys=sk, splits=ns, us=round(t, 2),
                 TBps=round(gb / t * 1e3, 2))


def attn2_bench():
    """In-graph decode attention at the engine's shapes."""
    H, Hkv, D, blk = 32, 8, 128, 16
    for B, ctx, qlen in ((8, 500, 1), (8, 500, 4), (8, 900, 1)):
        nb = (1024 + blk - 1) // blk
        kc = torch.randn(B * nb, Hkv, blk, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn_like(kc)
        bt = torch.arange(B * nb, dtype=torch.int32, device=dev).view(B, -1)
        Tq = B * qlen
        q = torch.randn(max(16, Tq), H * D, device=dev, dtype=torch.bfloat16)
        cu = torch.arange(0, Tq + 1, qlen, dtype=torch.int32, device=dev)
        cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        ws = ops.AttnWorkspace(dev, 256, H, D, 32)
        gb = 2 * B * ctx * Hkv * D * 2 / 1e9
        for sk, ns in ((128, 8), (128, (ctx + 127) // 128), (256, 4), (64, 16)):
            t = gtime(lambda: ops.attention(q, kc, vc, cu, n_heads=H, n_kv=Hkv, head_dim=D,
                                            causal=True, max_q=qlen, ctx_lens=cl, block_tables=bt,
                                            grouped=True, split_keys=sk, num_splits=ns,
                                            workspace=ws))
            emit(kernel="decode_attn_graph", B=B, ctx=ctx, qlen=qlen, split_keys=sk, splits=ns,
                 us=round(t, 2), TBps=round(gb / t * 1e3, 2))
    # whisper-large cross-attention (contiguous encoder rows) and self-attention
    Hw, Dw, T = 20, 64, 1500
    B = 8
    enc = torch.randn(B * T, 2 * Hw * Dw, device=dev, dtype=torch.bfloat16)
    q = torch.randn(16, Hw * Dw, device=dev, dtype=torch.bfloat16)
    cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
    starts = torch.arange(0, B * T, T, dtype=torch.int32, device=dev)
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    ws = ops.AttnWorkspace(dev, 256, Hw, Dw, 32)
    for sk in (128, 256, 384, 512):
        ns = (T + sk - 1) // sk
        t = gtime(lambda: ops.attention(q, enc, enc[:, Hw * Dw:], cu, n_heads=Hw, n_kv=Hw,
                                        head_dim=Dw, causal=False, max_q=1, cu_k=starts,
                                        ctx_lens=lens, grouped=True, split_keys=sk, num_splits=ns,
                                        workspace=ws))
        emit(kernel="whisper_cross_graph", B=B, split_keys=sk, splits=ns, us=round(t, 2),
             TBps=round(2 * B * T * Hw * Dw * 2 / 1e9 / t * 1e3, 2))


def tiny_bench():
    """Floor of a graph-replayed tiny kernel."""
    x = torch.zeros(16, 4096, device=dev, dtype=torch.bfloat16)
    emit(kernel="graph_tiny_add", us=round(gtime(lambda: x.add_(1)), 2))
    part = torch.randn(8, 16, 4096, device=dev)
    res = torch.randn(16, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.ones(4096, device=dev, dtype=torch.bfloat16)
    emit(kernel="graph_slab_rmsnorm_S8", us=round(gtime(lambda: ops.slab_rmsnorm(part, res, w, 1e-5)), 2))
    gu = torch.randn(8, 16, 2 * 14336, device=dev)
    emit(kernel="graph_slab_silu_S8", us=round(gtime(lambda: ops.slab_silu_mul(gu)), 2))
    for name, (N, K) in {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
                         "down": (4096, 14336)}.items():
        wp = ops.shuffle_weight(torch.randn(N, K, device=dev, dtype=torch.bfloat16))
        xx = torch.randn(16, K, device=dev, dtype=torch.bfloat16)
        res = {"kernel": "graph_gemm", "shape": name}
        for S in (1, 2, 4, 8):
            if K % (S * 128):
                continue
            t = gtime(lambda: ops.skinny_gemm(xx, wp, S), inner=10)
            res[f"S{S}_us"] = round(t, 2)
            res[f"S{S}_TBps"] = round(N * K * 2 / 1e9 / t * 1e3, 2)
        emit(**res)
        del wp


def fused_bench():
    """Fused-epilogue decode GEMMs vs plain skinny GEMM at each split, graph-timed
    on COLD weights: the graph cycles through enough weight copies (>= 1 GB) that
    no call finds its weight in the 256 MB Infinity Cache, as in a real decode
    step that streams the whole model."""
    scr = ops.FusedScratch(dev)
    M, d, H, Hkv, D, blk = 16, 4096, 32, 8, 128, 16
    pos = torch.arange(M, dtype=torch.int32, device=dev) + 100
    cs = torch.randn(4096, D // 2, 2, device=dev)
    kc = torch.zeros(64, Hkv, blk, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    slots = torch.arange(M, dtype=torch.int32, device=dev)
    q = torch.empty(M, H * D, device=dev, dtype=torch.bfloat16)
    for name, (N, K), mode, rows in (("qkv", (6144, 4096), "rope", 128),
                                     ("o", (4096, 4096), "resid", 0),
                                     ("gate_up", (28672, 4096), "silu", 256),
                                     ("down", (4096, 14336), "resid", 0)):
        ncopy = max(2, -(-(1 << 30) // (N * K * 2)))
        base = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        wps = [ops.shuffle_weight(base) for _ in range(ncopy)]
        del base
        xx = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        res_ = torch.randn(M, N if mode == "resid" else d, device=dev, dtype=torch.bfloat16)
        if rows:
            scr.rowsq[: rows * M].fill_(float(K) / rows)
        gb = N * K * 2 / 1e9
        res = {"kernel": "graph_fused_cold", "shape": name, "mode": mode, "copies": ncopy}
        for S in (1, 2, 4, 8):
            if K % (S * 128):
                continue
            kw = dict(splits=S, rt=1)
            if mode == "rope":
                kw.update(norm=True, rowsq_tiles=rows, positions=pos, cos_sin=cs, q_out=q,
                          k_cache=kc, v_cache=vc, slots=slots, n_heads=H, n_kv=Hkv, head_dim=D)
            elif mode == "silu":
                kw.update(norm=True, rowsq_tiles=rows)
            else:
                kw.update(residual=res_)
            it = iter(range(1 << 30))

            def fused():
                ops.skinny_fused(xx, wps[next(it) % ncopy], mode, scr, **kw)

            def plain():
                ops.skinny_gemm(xx, wps[next(it) % ncopy], S)
            t = gtime(fused, inner=2 * ncopy)
            res[f"fusedS{S}_us"] = round(t, 2)
            if S == 1 and N % 128 == 0:
                for rt4 in (1, 2):
                    kw1 = dict(kw, wr=4, rt=rt4)

                    def fused4():
                        ops.skinny_fused(xx, wps[next(it) % ncopy], mode, scr, **kw1)
                    t4 = gtime(fused4, inner=2 * ncopy)
                    res[f"fusedS1wr4rt{rt4}_us"] = round(t4, 2)
            res[f"fusedS{S}_TBps"] = round(gb / t * 1e3, 2)
            res[f"plainS{S}_us"] = round(gtime(plain, inner=2 * ncopy), 2)
        emit(**res)
        del wps


def fused70_bench():
    """Llama-3-70B decode GEMM shapes (d 8192, ffn 28672, 64/8 heads) on the
    fused kernel, every (split, tile rows, waves-along-rows) layout, cold
    weights (copies cycled); ``units`` = workgroups before the co-scheduling cap."""
    M = int(os.environ.get("KB_M", "16"))
    scr = ops.FusedScratch(dev)
    d, H, Hkv, D, blk = 8192, 64, 8, 128, 16
    pos = torch.arange(M, dtype=torch.int32, device=dev) + 100
    cs = torch.randn(4096, D // 2, 2, device=dev)
    kc = torch.zeros(64, Hkv, blk, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    slots = torch.arange(M, dtype=torch.int32, device=dev)
    q = torch.empty(M, H * D, device=dev, dtype=torch.bfloat16)
    rows = d // 32
    for name, (N, K), mode in (("qkv", (10240, 8192), "rope"), ("o", (8192, 8192), "resid"),
                               ("gate_up", (57344, 8192), "silu"), ("down", (8192, 28672), "resid")):
        ncopy = max(2, -(-(3 << 30) // (N * K * 2)))
        base = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        wps = [ops.shuffle_weight(base) for _ in range(ncopy)]
        del base
        xx = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        res_ = torch.randn(M, N if mode == "resid" else d, device=dev, dtype=torch.bfloat16)
        scr.rowsq[: rows * M].fill_(float(K) / rows)
        gb = N * K * 2 / 1e9
        res = {"kernel": "graph_fused_cold_70b", "M": M, "shape": name, "mode": mode, "GB": round(gb, 3)}
        for S in (1, 2, 4):
            for rt in ((1, 2, 4) if M == 64 else (1, 2)):
                for wr in (1, 4):
                    if K % (S * 128) or (wr == 4 and S != 1) or N % (16 * rt * wr):
                        continue
                    kw = dict(splits=S, rt=rt, wr=wr)
                    if mode == "rope":
                        kw.update(norm=True, rowsq_tiles=rows, positions=pos, cos_sin=cs, q_out=q,
                                  k_cache=kc, v_cache=vc, slots=slots, n_heads=H, n_kv=Hkv,
                                  head_dim=D)
                    elif mode == "silu":
                        kw.update(norm=True, rowsq_tiles=rows)
                    else:
                        kw.update(residual=res_)
                    it = iter(range(1 << 30))

                    def fused():
                        ops.skinny_fused(xx, wps[next(it) % ncopy], mode, scr, **kw)
                    t = gtime(fused, inner=2 * ncopy)
                    units = (N // (16 * rt * wr)) * S
                    res[f"S{S}rt{rt}wr{wr}_u{units}"] = [round(t, 2), round(gb / t * 1e3, 2)]
        emit(**res)
        del wps


def stream_bench():
    """HBM read roofline of this box: torch sum over a 2 GB bf16 buffer."""
    buf = torch.ones(1 << 30, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: buf.sum(dtype=torch.float32), reps=10)
    emit(kernel="stream_sum_2GB", us=round(t, 2), TBps=round(2.0 * (1 << 30) / 1e6 / t, 2))
    del buf


def slab_bench():
    for M, d, S in ((16, 4096, 4), (16, 4096, 2), (32, 4096, 4)):
        part = torch.randn(S, M, d, device=dev)
        res = torch.randn(M, d, device=dev, dtype=torch.bfloat16)
        w = torch.ones(d, device=dev, dtype=torch.bfloat16)
        emit(kernel="slab_rmsnorm", M=M, d=d, S=S,
             us=round(timeit(lambda: ops.slab_rmsnorm(part, res, w, 1e-5)), 2))
    part = torch.randn(1, 16, 2 * 14336, device=dev)
    emit(kernel="slab_silu_mul", M=16, F=14336, S=1, us=round(timeit(lambda: ops.slab_silu_mul(part)), 2))
    x = torch.randn(16, 4096, device=dev, dtype=torch.bfloat16)
    emit(kernel="rmsnorm", M=16, d=4096, us=round(timeit(lambda: ops.rmsnorm(x, w, 1e-5)), 2))
    emit(kernel="empty_torch_add", us=round(timeit(lambda: x.add_(0)), 2))


if __name__ == "__main__":
    which = sys.argv[1:] or ["gemm", "attn", "slab"]
    if "attn2" in which:
        attn2_bench()
    if "tiny" in which:
        tiny_bench()
    if "fused" in which:
        fused_bench()
    if "fused70" in which:
        fused70_bench()
    if "stream" in which:
        stream_bench()
    if "gemm" in which:
        gemm_bench()
    if "attn" in which:
        attn_bench()
    if "slab" in which:
        slab_bench()
