"""Split-K tiled GEMM (ops.gemm_sk) vs hipBLASLt (torch.matmul) on the prefill
and Whisper-encoder projection shapes, cold weights (a ring of weight copies
larger than the 256 MiB Infinity Cache), CUDA-event timing; prints one JSON
line per (shape, variant) and the planner's pick.

    python scripts/exp/gemm_sk_bench.py [--ms 300,600,1200] [--grid]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from loqa_hub_amd import ops  # noqa: E402

LLAMA = {"qkv": (6144, 4096, "bf16"), "o": (4096, 4096, "resid"), "gu": (28672, 4096, "swiglu"),
         "down": (4096, 14336, "resid")}
# Llama-3-70B TP=8 rank shards (config 5 prompt passes; o / down are partials
# for the all-reduce, plain bf16 outputs)
TP70 = {"qkv70": (1280, 8192, "bf16"), "o70": (8192, 1024, "bf16"), "gu70": (7168, 8192, "swiglu"),
        "down70": (8192, 3584, "bf16")}
WHISPER = {"enc_qkv": (3840, 1280, "bf16"), "enc_o": (1280, 1280, "resid"),
           "enc_fc1": (5120, 1280, "bf16"), "enc_fc2": (1280, 5120, "resid")}


def timeit(fn, n_w, iters=30):
    for i in range(3):
        fn(i % n_w)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n_w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="300,600,1200")
    ap.add_argument("--wms", default="1500,3000,6000")
    ap.add_argument("--grid", action="store_true", help="time every (layout, S)")
    ap.add_argument("--only", default="", help="comma list of shape names")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cases = [(m, k, v) for m in map(int, a.ms.split(",")) for k, v in LLAMA.items()]
    cases += [(m, k, v) for m in map(int, a.wms.split(",")) for k, v in WHISPER.items()]
    cases += [(m, k, v) for m in map(int, a.ms.split(",")) for k, v in TP70.items()]
    if a.only:
        cases = [c for c in cases if c[1] in a.only.split(",")]
    for M, name, (N, K, epi) in cases:
        wbytes = N * K * 2
        n_w = max(2, (768 << 20) // wbytes)
        ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(n_w)]
        x = torch.randn(M, K, device=dev).bfloat16()
        res = torch.randn(M, N, device=dev).bfloat16()
        flops = 2.0 * M * N * K
        t_blas = timeit(lambda i: torch.matmul(x, ws[i].t()), n_w)
        lay, s = ops.gemm_sk_plan(M, N, K, epi)

        def run(i, lay=lay, s=s):
            if epi == "resid":
                ops.gemm_sk(x, ws[i], epi="resid", residual=res, layout=lay, splits=s)
            else:
                ops.gemm_sk(x, ws[i], epi=epi, layout=lay, splits=s)
        t_plan = timeit(run, n_w)
        ws_t = {}
        for depth in ((0, 1) if N % 128 == 0 else ()):
            def run_ws(i, depth=depth):
                if epi == "resid":
                    ops.gemm_ws(x, ws[i], epi="resid", residual=res, depth=depth)
                else:
                    ops.gemm_ws(x, ws[i], epi=epi, depth=depth)
            ws_t[depth] = round(timeit(run_ws, n_w), 1)
        out = {"shape": name, "M": M, "N": N, "K": K, "epi": epi, "hipblaslt_us": round(t_blas, 1),
               "ws_us": ws_t,
               "hipblaslt_pf": round(flops / t_blas / 1e9, 3), "plan": [lay, s],
               "plan_us": round(t_plan, 1), "plan_pf": round(flops / t_plan / 1e9, 3)}
        if a.grid:
            best = None
            grid = {}
            for l2 in sorted(ops.SK_LAYOUTS):
                bn, bm = ops.SK_LAYOUTS[l2][:2]
                if N % bn:
                    continue
                for s2 in (1, 2, 3, 4, 6, 8):
                    if s2 > K // 64 or (s2 > 1 and K // 64 // s2 < 4):
                        continue
                    t = timeit(lambda i, l2=l2, s2=s2: run(i, l2, s2), n_w, iters=15)
                    grid[f"{l2},{s2}"] = round(t, 1)
                    if best is None or t < best[2]:
                        best = (l2, s2, t)
            out["best"] = [best[0], best[1], round(best[2], 1)]
            out["best_pf"] = round(flops / best[2] / 1e9, 3)
            out["grid"] = grid
        print(json.dumps(out), flush=True)
        del ws


if __name__ == "__main__":
    main()
