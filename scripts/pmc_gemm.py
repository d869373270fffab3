"""The four Llama-3-8B decode GEMMs of a fused decode step (qkv with the
RMSNorm prologue + RoPE / paged-KV epilogue, o + residual, gate|up + SiLU, down
+ residual; Mpad 16, the layouts the serving tuner picks), each run ALONE and
repeatedly on cold weights (enough copies to outgrow the 256 MiB Infinity
Cache), for hardware counters: run under ``rocprofv3 --pmc`` and reduce with
``scripts/pmc_summary.py --shapes <this script's JSON>``.

In the served pipeline the counters of a kernel are polluted by whatever runs
concurrently on the other decoder's stream (the TCC read counters are per
device, not per dispatch), so the bench-wide PMC table cannot give a kernel's
own HBM bytes; here nothing else runs. The JSON written to ``--shapes`` maps
each dispatch's (kernel template, grid threads) to its label and ALGORITHMIC
bytes (weights + activations + outputs), printed beside the counter bytes.

    python scripts/pmc_gemm.py --shapes gpurun_out/pmc_gemm_shapes.json [--reps 40]
"""
import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from loqa_hub_amd import ops  # noqa: E402
from loqa_hub_amd.ops import reference as ref  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", required=True)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--model", default="llama3-8b")
    a = ap.parse_args()
    from loqa_hub_amd.models.configs import llama_config
    cfg = llama_config(a.model)
    dev = torch.device("cuda", 0)
    bf = dict(dtype=torch.bfloat16, device=dev)
    torch.manual_seed(0)
    H, Hkv, D, d, F = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.d_model, cfg.ffn_dim
    Mpad = 16
    scr = ops.FusedScratch(dev)
    tiles = d // 32
    norm_w = torch.ones(d, **bf)
    kc = torch.zeros(8, Hkv, 16, D, **bf)
    pos = torch.arange(Mpad, dtype=torch.int32, device=dev)
    wqkv = torch.randn((H + 2 * Hkv) * D, d, **bf) * 0.02
    wgu = torch.randn(2 * F, d, **bf) * 0.02
    shapes = {
        "qkv": (ops.FusedLinear(wqkv, norm="rms", norm_w=norm_w, perm=ref.perm_rope_qkv(H, Hkv, D).to(dev)),
                "rope", dict(rowsq_tiles=tiles, positions=pos, cos_sin=None,
                             q_out=torch.empty(Mpad, H * D, **bf), k_cache=kc,
                             v_cache=torch.zeros_like(kc), slots=pos, n_heads=H, n_kv=Hkv, head_dim=D),
                dict(heads=(H, Hkv, D), norm="rms")),
        "o": (ops.FusedLinear(torch.randn(d, H * D, **bf) * 0.02), "resid",
              dict(residual=torch.zeros(Mpad, d, **bf)), {}),
        "gate_up": (ops.FusedLinear(wgu, norm="rms", norm_w=norm_w, perm=ref.perm_gate_up(F).to(dev)),
                    "silu", dict(rowsq_tiles=tiles), dict(norm="rms")),
        "down": (ops.FusedLinear(torch.randn(d, F, **bf) * 0.02), "resid",
                 dict(residual=torch.zeros(Mpad, d, **bf)), {}),
    }
    scr.rowsq[: tiles * Mpad].fill_(float(d) / tiles)
    out = []
    for name, (lin, mode, kw, tkw) in shapes.items():
        # the serving tuner's layout for this shape (same cap, cold weights)
        ops.tune_fused(lin, mode, mpads=(Mpad,), **tkw)
        S, rt, wr = ops._FSPLITS[(mode, lin.N, lin.K, Mpad)][:3]
        wgs = (lin.N // (16 * rt * wr)) * S
        wbytes = lin.N * lin.K * 2
        xbytes = Mpad * lin.K * 2
        obytes = {"rope": Mpad * lin.N * 2, "resid": 2 * Mpad * lin.N * 2,
                  "silu": Mpad * lin.N}[mode]
        nbytes = wbytes + xbytes + obytes
        copies = [lin]
        for _ in range(min(15, -(-(768 << 20) // wbytes) - 1)):
            c = copy.copy(lin)
            c.wp = lin.wp.clone()
            copies.append(c)
        x = torch.randn(Mpad, lin.K, **bf)
        torch.cuda.synchronize()
        for i in range(a.reps):
            ops.skinny_fused(x, copies[i % len(copies)], mode, scr, splits=S, rt=rt, wr=wr, **kw)
        torch.cuda.synchronize()
        out.append({"label": name, "mode": mode, "grid": wgs * 256, "algorithmic_bytes": nbytes,
                    "weight_bytes": wbytes, "layout": [S, rt, wr], "workgroups": wgs})
        print(json.dumps(out[-1]), flush=True)
    with open(a.shapes, "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
